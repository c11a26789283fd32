# The zipf-ckpt two-process case under the engine's A/B switches; an assertion failure (pytest
# exit 1) moves on to the next variant, anything else (a crash, a time limit) ends the run.
O=gpurun_out/$1
mkdir -p $O
for V in default FG_NARROW_TABLES=0 FG_TILE_SPLIT=0 FG_TILE_STATE=0; do
  if [ $V = default ]; then E=""; else E="$V"; fi
  env $E timeout -k 10 200 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider \
      "tests/test_gpu_multiproc.py::test_two_processes_two_phase_hip_path_matches_oracle[zipf-ckpt]" > $O/$V.log 2>&1
  rc=$?
  echo "$V rc=$rc"; grep -E "missing|extra|rows per|passed|failed" $O/$V.log | grep -v "^\[" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

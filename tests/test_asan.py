"""The engine's host logic under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU.

flink_amd/Makefile `asan` builds libflinkgpu_asan.so: fg_engine.cpp and the key dictionary's
host code instrumented (-Xarch_host -fsanitize=address,undefined; device code is not), linked
with the regular kernel objects. tests/asan/abi_driver.c drives every C-ABI path that needs no
device -- the reference's window-spec validation messages (the golden error vectors of
tests/golden/assigner_cases.json), NULL-handle and argument checks, the BinaryRowData hash
against the oracle's restatement -- and fg_open of valid specs, which fails with FG_EDEVICE
without a GPU. A sanitizer report fails the test (the driver aborts on the first one). (The
round-4 build of this found fg_open writing through a NULL handle pointer.)"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = "/opt/rocm/lib/llvm/lib/clang"
KIND = {"tumble": 0, "hop": 1, "cumulate": 2}


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "flink_amd"), "asan"], check=True)
    rt = sorted(d for d in os.listdir(RT))[-1]
    rtdir = os.path.join(RT, rt, "lib", "linux")
    exe = os.path.join(ROOT, "flink_amd", "build_asan", "abi_driver")
    subprocess.run(["/opt/rocm/lib/llvm/bin/clang", "-O1", "-g", "-fsanitize=address,undefined", "-shared-libsan",
                    "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "asan", "abi_driver.c"), "-L" + os.path.join(ROOT, "flink_amd"),
                    "-lflinkgpu_asan", "-Wl,-rpath," + os.path.join(ROOT, "flink_amd"), "-Wl,-rpath," + rtdir, "-o", exe],
                   check=True)
    return exe


@pytest.mark.skipif(not os.path.isdir(RT), reason="ROCm clang (ASan runtime) not present")
def test_host_logic_under_asan_ubsan(oracle_mod):
    exe = _build()
    lines = []
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "assigner_cases.json")))
    for e in golden["errors"]:
        c = e["config"]
        cs = 0 if c.get("count_star_index", 0) < 0 else 1
        lines.append(f"spec {KIND[c['kind']]} {c['size']} {c['slide']} {c['offset']} 0 {cs} 1 {e['message']}")
    for kind, size, slide in (("tumble", 1000, 0), ("hop", 5000, 1000), ("cumulate", 3_600_000, 60_000)):
        lines.append(f"spec {KIND[kind]} {size} {slide} 0 0 1 0 -")
        lines.append(f"spec {KIND[kind]} {size} {slide} 0 1 1 {1 if kind == 'cumulate' else 0} -")   # DataStream
    rng = np.random.default_rng(3)
    for n in (8, 16, 24, 40, 64, 256):
        row = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        lines.append(f"hash {row.hex()} {oracle_mod.binaryrow_hash_bytes(row)}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    p = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300, env=env)
    out = p.stdout + p.stderr
    assert "Sanitizer" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    assert f"{len(lines)} cases, 0 failures" in p.stdout, out[-2000:]

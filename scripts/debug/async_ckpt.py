"""A/B of the CUMULATE checkpoint/restore async case: synchronous vs async watermarks."""
import os, sys, traceback
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O
O.build()
from tests.test_gpu_async import _run, _cfg
for sync in (True, False):
    for ck in (4, 8):
        try:
            _run(O, _cfg("cumulate"), jitter=1500, delay=300, ckpt_every=ck, collect_every=2, sync=sync)
            print("sync", sync, "ckpt_every", ck, "OK", flush=True)
        except AssertionError as e:
            print("sync", sync, "ckpt_every", ck, "FAIL", str(e).splitlines()[0], flush=True)

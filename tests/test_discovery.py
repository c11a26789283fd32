"""AMD GPU discovery script: output contract of the reference's
GPUDriver discovery scripts, with a stand-in rocm-smi on PATH (no GPU needed)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "flink_amd", "discovery", "amd-gpu-discovery.sh")


def fake_smi(tmp_path, cards=8):
    """`rocm-smi --showid --csv` as ROCm 7.2 prints it on an MI355X box (captured there:
    profiles/r02/discovery/rocm_smi_showid.csv): a power-state warning, a blank line, the
    CSV header, one `cardN,...` row per GPU."""
    p = tmp_path / "rocm-smi"
    rows = "\\n".join(f"card{i},N/A,0x75a3,0x00,0x75a3,{24656 + i}" for i in range(cards))
    p.write_text("#!/bin/sh\nprintf 'WARNING: AMD GPU device(s) is/are in a low-power state. Check power "
                 "control/runtime_status\\n\\ndevice,Device Name,Device ID,Device Rev,Subsystem ID,GUID\\n"
                 f"{rows}\\n'\n")
    p.chmod(0o755)
    return str(p)


def run(args, smi, env_extra=None):
    env = dict(os.environ, ROCM_SMI=smi)
    env.update(env_extra or {})
    r = subprocess.run(["bash", SCRIPT] + args, capture_output=True, text=True, env=env)
    return r.returncode, r.stdout.strip()


def test_lists_requested_amount(tmp_path):
    smi = fake_smi(tmp_path)
    assert run(["2"], smi) == (0, "0,1")
    assert run(["8"], smi) == (0, "0,1,2,3,4,5,6,7")
    assert run(["0"], smi) == (0, "")
    assert run(["9"], smi)[0] == 1      # fewer GPUs than requested


def test_coordination_mode_gives_disjoint_sets(tmp_path):
    smi = fake_smi(tmp_path, cards=4)
    f = str(tmp_path / "coord")
    alive = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        rc1, a = run(["2", "--enable-coordination-mode", "--coordination-file", f], smi, {"FLINK_TM_PID": str(alive.pid)})
        rc2, b = run(["2", "--enable-coordination-mode", "--coordination-file", f], smi, {"FLINK_TM_PID": str(alive.pid)})
        rc3, c = run(["1", "--enable-coordination-mode", "--coordination-file", f], smi, {"FLINK_TM_PID": str(alive.pid)})
        assert (rc1, rc2, rc3) == (0, 0, 1)
        assert set(a.split(",")).isdisjoint(b.split(",")) and len(set(a.split(",") + b.split(","))) == 4
    finally:
        alive.kill()
        alive.wait()
    # the owner is gone: its claims are released
    rc, d = run(["4", "--enable-coordination-mode", "--coordination-file", f], smi, {"FLINK_TM_PID": "1"})
    assert rc == 0 and d == "0,1,2,3"


@pytest.mark.gpu
def test_real_rocm_smi_lists_the_visible_gpus():
    """On the GPU box: the script parses the real `rocm-smi --showid --csv` and lists as many
    indices as HIP sees, each a valid HIP ordinal (the box exposes its card as card0 with
    HIP_VISIBLE_DEVICES=0; profiles/r02/discovery/)."""
    import shutil

    import torch
    if shutil.which("rocm-smi") is None:
        pytest.skip("no rocm-smi")
    n = torch.cuda.device_count()
    if n == 0:
        pytest.skip("no GPU visible")
    env = dict(os.environ)
    env.pop("ROCM_SMI", None)
    r = subprocess.run(["bash", SCRIPT, str(n)], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    idx = [int(x) for x in r.stdout.strip().split(",")]
    assert len(idx) == n and all(0 <= i < n for i in idx)

"""AMD GPU discovery script: output contract of the reference's
GPUDriver discovery scripts, with a stand-in rocm-smi on PATH (no GPU needed)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "flink_amd", "discovery", "amd-gpu-discovery.sh")


def fake_smi(tmp_path, cards=8):
    p = tmp_path / "rocm-smi"
    rows = "\\n".join(f"card{i},0x75a3" for i in range(cards))
    p.write_text(f"#!/bin/sh\nprintf 'device,GPU ID\\n{rows}\\n'\n")
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

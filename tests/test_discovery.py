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
    env = dict(os.environ, ROCM_SMI=smi, HIP_BUS_IDS="/nonexistent")   # (card indices as they are)
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


def fake_smi_with_bus(tmp_path, buses):
    """rocm-smi answering --showid and --showbus (`card<i>,<PCI bus>` rows, as captured in
    profiles/r02/discovery/rocm_smi_showbus.csv)."""
    p = tmp_path / "rocm-smi"
    ids = "\\n".join(f"card{i},N/A,0x75a3,0x00,0x75a3,{24656 + i}" for i in range(len(buses)))
    bus = "\\n".join(f"card{i},{b}" for i, b in enumerate(buses))
    p.write_text("#!/bin/sh\nif [ \"$1\" = --showbus ]; then printf 'device,PCI Bus\\n" + bus + "\\n'; "
                 "else printf 'device,Device Name,Device ID,Device Rev,Subsystem ID,GUID\\n" + ids + "\\n'; fi\n")
    p.chmod(0o755)
    return str(p)


def test_cards_map_to_hip_ordinals_by_pci_bus(tmp_path):
    """rocm-smi numbers the host's cards, HIP only the visible devices in its own order: the
    script maps each card to the HIP ordinal of the same PCI bus id (hip-pci-bus-ids) and
    leaves out the cards HIP does not see."""
    smi = fake_smi_with_bus(tmp_path, ["0000:0D:00.0", "0000:1A:00.0", "0000:8F:00.0", "0000:9C:00.0"])
    tool = tmp_path / "busids"
    tool.write_text("#!/bin/sh\nprintf '0 0000:8f:00.0\\n1 0000:0d:00.0\\n'\n")   # HIP sees cards 2 and 0
    tool.chmod(0o755)
    env = {"HIP_BUS_IDS": str(tool)}
    assert run(["2"], smi, env) == (0, "1,0")        # card0 -> ordinal 1, card2 -> ordinal 0
    assert run(["3"], smi, env)[0] == 1              # only two cards are visible to HIP


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


@pytest.mark.gpu
def test_real_bus_id_map_matches_hip():
    """On the GPU box: hip-pci-bus-ids lists every HIP ordinal with its bus id, and the card the
    script maps to ordinal i has that bus id in `rocm-smi --showbus`."""
    import shutil
    tool = os.path.join(ROOT, "flink_amd", "discovery", "hip-pci-bus-ids")
    if shutil.which("rocm-smi") is None or not os.path.exists(tool):
        pytest.skip("no rocm-smi or bus-id tool")
    hip = dict(ln.split() for ln in subprocess.run([tool], capture_output=True, text=True, check=True).stdout.split("\n")
               if ln.strip())
    bus = subprocess.run(["rocm-smi", "--showbus", "--csv"], capture_output=True, text=True).stdout
    cards = {ln.split(",")[1].strip().lower() for ln in bus.splitlines() if ln.startswith("card")}
    assert hip and all(b in cards for b in hip.values()), (hip, cards)
    env = dict(os.environ)
    env.pop("ROCM_SMI", None)
    r = subprocess.run(["bash", SCRIPT, str(len(hip))], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    assert sorted(r.stdout.strip().split(",")) == sorted(hip)

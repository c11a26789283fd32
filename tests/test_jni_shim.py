"""The Java shim + JNI glue (java/, jni/) against the C-ABI they bind, without a JDK (none in this
image): the fg_config image FgConfig.java writes has the C struct's layout and
enum values, and every native FlinkGpu.java declares has its JNIEXPORT in jni/flink_gpu_jni.c
(same name, same argument count, calling the C-ABI entry point it names). The glue itself is
compiled against a stub <jni.h> (tests/jni_stub) and driven through a fake JNIEnv: its exceptions
on the CPU, and (gpu) a tiny job whose fired columns are read as host memory."""
import ctypes as C
import json
import os
import re
import subprocess

import numpy as np
import pytest

from flink_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "main", "java", "org", "apache", "flink", "table", "runtime", "operators",
                    "window", "gpu")
JNI_C = os.path.join(ROOT, "jni", "flink_gpu_jni.c")


def _java_consts():
    src = open(os.path.join(JAVA, "FgConfig.java")).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"public static final int (\w+) = (-?\d+);", src)}


def test_config_image_matches_c_layout():
    k = _java_consts()
    for name, _ in L.FgConfig._fields_:
        assert k[name.upper()] == getattr(L.FgConfig, name).offset, name
    assert k["SIZE"] == C.sizeof(L.FgConfig)
    assert k["MAX_AGGS"] == 8


def test_enum_values_match_header():
    k = _java_consts()
    for name in ("MODE_SQL", "MODE_DATASTREAM", "TUMBLE", "HOP", "CUMULATE", "VAL_NONE", "VAL_I64", "VAL_F64",
                 "AGG_COUNT_STAR", "AGG_COUNT", "AGG_SUM", "AGG_AVG", "AGG_SUM0", "AGG_MIN", "AGG_MAX",
                 "FLAG_LOCAL_PARTIALS", "FLAG_PROCTIME", "FLAG_WINDOWED", "FLAG_PURGING_TRIGGER"):
        assert k[name] == getattr(L, name), name


def _java_natives():
    src = open(os.path.join(JAVA, "FlinkGpu.java")).read()
    out = {}
    for m in re.finditer(r"public static native \w+(?:\[\])? (\w+)\(([^)]*)\);", src, re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args)
    return out


def _jni_exports():
    src = open(JNI_C).read()
    out = {}
    for m in re.finditer(r"JNIEXPORT \w+ JNICALL FN\((\w+)\)\(([^)]*)\)", src, re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args) - 2   # JNIEnv*, jclass
    return out


def test_every_native_has_its_jni_export():
    nat, exp = _java_natives(), _jni_exports()
    assert nat and set(nat) == set(exp), (sorted(nat), sorted(exp))
    for name, n in nat.items():
        assert exp[name] == n, f"{name}: Java declares {n} arguments, the JNI export takes {exp[name]}"
    src = open(JNI_C).read()
    assert "#define FN(name) Java_org_apache_flink_table_runtime_operators_window_gpu_FlinkGpu_##name" in src


def test_jni_calls_only_declared_entry_points():
    header = open(os.path.join(ROOT, "include", "flinkgpu.h")).read()
    declared = set(re.findall(r"\b(fg_\w+)\s*\(", header))
    called = set(re.findall(r"\b(fg_\w+)\s*\(", open(JNI_C).read()))
    assert called <= declared, called - declared
    for fn in ("fg_open", "fg_add_batch", "fg_add_rows", "fg_add_partials", "fg_advance_progress", "fg_flush",
               "fg_snapshot_state", "fg_restore", "fg_late_dropped", "fg_close", "fg_key_dict_intern"):
        assert fn in called, fn


def test_java_calls_only_declared_natives():
    """every FlinkGpu.x(...) call in the shim names a native FlinkGpu.java declares"""
    nat = _java_natives()
    root = os.path.join(ROOT, "java", "src", "main", "java")
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith(".java") and f != "FlinkGpu.java":
                for m in re.finditer(r"FlinkGpu\.(\w+)\(", open(os.path.join(dirpath, f)).read()):
                    assert m.group(1) in nat, f"{f}: FlinkGpu.{m.group(1)} is not a native"


STUB = os.path.join(ROOT, "tests", "jni_stub")


def _build_jni_driver(tmp_path):
    """jni/flink_gpu_jni.c + tests/jni_stub/jni_driver.c against the stub <jni.h>, warnings as
    errors, linked with the in-tree libflinkgpu.so"""
    exe = str(tmp_path / "jni_driver")
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-I" + STUB, "-I" + os.path.join(ROOT, "include"),
                    JNI_C, os.path.join(STUB, "jni_driver.c"), "-L" + os.path.join(ROOT, "flink_amd"), "-lflinkgpu",
                    "-Wl,-rpath," + os.path.join(ROOT, "flink_amd"), "-o", exe], check=True)
    return exe


def test_jni_glue_errors_through_fake_jnienv(tmp_path):
    """the glue's exceptions, driven as a JVM would: the reference's window-spec messages as
    IllegalArgumentException (golden error vectors), heap buffers refused, zone-rule array checks,
    and a valid spec -> a handle (GPU host) or RuntimeException (no device)"""
    exe = _build_jni_driver(tmp_path)
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "assigner_cases.json")))
    kind = {"tumble": 0, "hop": 1, "cumulate": 2}
    lines = []
    for e in golden["errors"]:
        c = e["config"]
        cs = 0 if c.get("count_star_index", 0) < 0 else 1
        lines.append(f"spec {kind[c['kind']]} {c['size']} {c['slide']} {c['offset']} {cs} {e['message']}")
    p = subprocess.run([exe, "errors"], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert f"{len(lines) + 5} cases, 0 failures" in p.stdout, p.stdout


@pytest.mark.gpu
def test_jni_glue_on_gpu_host_columns(tmp_path):
    """open / addBatch / advanceProgressAsync + collectFired / snapshotStateAsync / advanceProgress /
    snapshotStateWait / flushPartials through the glue on the GPU: the driver reads every fired column on the HOST (the direct
    buffers a JVM would read), totals against numpy; then the two-phase edge through the comm
    natives at world size 1 (commUniqueId / commOpen / commExchangeFired over RCCL): the global
    handle fires what the single-phase operator fired"""
    exe = _build_jni_driver(tmp_path)
    p = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "gpu done" in p.stdout, p.stdout + p.stderr
    out = {ln.split()[0]: ln.split()[1:] for ln in p.stdout.splitlines() if ln}
    i = np.arange(1000)
    key, rt, val = i % 10, 5 * i, 1.0 + i % 3

    def expect(sel):
        we = (rt[sel] // 1000 + 1) * 1000
        pairs = set(zip(key[sel], we))
        return (len(pairs), int(sel.sum()), float(val[sel].sum()), sum(k for k, _ in pairs), sum(w for _, w in pairs))

    assert out["comm_wm"] == ["2999", "sent", "0"]   # (world size 1: nothing leaves the rank)
    # the round form (ABI 16): watermark and epoch in-band, the rest of the windows merged into the global
    r = out["round_wm"]
    assert (r[0], r[2]) == ("10000", "7") and int(r[4]) == int(r[6]) > 0, r
    assert out["idle_wm"] == ["10001", "epoch", "8", "received", "0"], out["idle_wm"]
    for tag, sel in (("async", rt < 3000), ("sync", rt >= 3000), ("comm", rt < 3000), ("round", rt >= 3000)):
        f = out[tag]
        got = (int(f[1]), int(f[3]), float(f[5]), int(f[7]), int(f[9]))
        assert got == expect(sel), (tag, got, expect(sel))
    assert out["late"] == ["0"]
    # snapshotStateAsync after the 2999 watermark, collected after the 10000 advance fired the rest:
    # the image holds the state as of the async call -- the 400 records (10 keys x 2 windows) of the
    # windows ending 4000 and 5000 -- and that call's timer watermark
    assert out["snapshot"] == ["entries", "20", "cnt_star", "400", "wm", "2999"], out["snapshot"]
    # its slices (fg_snapshot_slices): the two open windows' slices, 10 keys each, both new (changed)
    assert out["slices"] == ["2", "first_end", "4000", "rows", "20", "changed", "2"], out["slices"]
    f = out["partials"]
    assert (int(f[1]), int(f[3]), int(f[5]), float(f[7])) == (50, 1000, 1000, float(val.sum()))


def test_fused_two_phase_operator_drives_the_rccl_edge():
    """The fused two-phase operator (GpuTwoPhaseWindowAggOperator) runs the keyBy edge over RCCL on
    the Flink path: it opens the communicator from the id its coordinator distributes and exchanges
    in rounds on its edge thread (ABI 16) -- the natives a Java operator must call for the edge to
    carry a job's partial rows instead of Netty. The incremental checkpoint reads the image's slices."""
    def calls(name):
        return set(re.findall(r"FlinkGpu\.(\w+)\(", open(os.path.join(JAVA, name)).read()))
    fused = calls("GpuTwoPhaseWindowAggOperator.java")
    for n in ("commUniqueId", "commOpen", "commRoundBegin", "commRoundExchange", "commRoundEnd", "commClose",
              "advanceProgressAsync", "collectFired", "snapshotStateAsync", "snapshotStateWait", "restore"):
        assert n in fused, n
    coord = open(os.path.join(JAVA, "GpuCommCoordinator.java")).read()
    assert "handleEventFromOperator" in coord and "failJob" in coord and "sendEvent" in coord
    fac = open(os.path.join(JAVA, "GpuTwoPhaseWindowAggOperatorFactory.java")).read()
    assert "CoordinatedOperatorFactory" in fac and "GpuCommCoordinator.Provider" in fac
    assert "snapshotSlices" in calls("GpuSlicingWindowProcessor.java")
    assert "snapshotSlices" in set(re.findall(r"FlinkGpu\.(\w+)\(", open(os.path.join(
        ROOT, "java", "src", "main", "java", "org", "apache", "flink", "streaming", "runtime", "operators",
        "windowing", "gpu", "GpuWindowOperator.java")).read()))

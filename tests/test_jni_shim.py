"""The Java shim + JNI glue (java/, jni/) against the C-ABI they bind, without a JDK (none in this
image): the fg_config image FgConfig.java writes has the C struct's layout and
enum values, and every native FlinkGpu.java declares has its JNIEXPORT in jni/flink_gpu_jni.c
(same name, same argument count, calling the C-ABI entry point it names)."""
import ctypes as C
import os
import re

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
                 "FLAG_LOCAL_PARTIALS", "FLAG_PROCTIME", "FLAG_WINDOWED"):
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

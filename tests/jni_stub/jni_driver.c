/*
 * Drives the exports of jni/flink_gpu_jni.c through a fake JNIEnv (tests/jni_stub/jni.h): what a
 * JVM would do through FlinkGpu.java's natives, in an image without a JDK. Test infrastructure
 * only (tests/test_jni_shim.py).
 *
 *   jni_driver errors   (stdin: "spec <kind> <size> <slide> <offset> <count_star 0/1> <message>")
 *       open() of each invalid window spec throws IllegalArgumentException with the reference's
 *       message; a heap (non-direct) buffer and mismatched zone-rule arrays throw
 *       IllegalArgumentException; a valid spec opens (GPU) or throws RuntimeException (no GPU)
 *   jni_driver gpu
 *       open / addBatch / advanceProgressAsync + collectFired / advanceProgress / flushPartials
 *       on a tiny TUMBLE job; the fired columns are read here, on the host (collectFired and
 *       flushPartials hand host memory to the JVM); prints the totals for the test to check
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"
#include "flinkgpu.h"

enum { K_CLASS, K_DIRECT, K_HEAP, K_OBJARR, K_LONGARR };
struct _jobject {
    int kind;
    void* addr;
    jlong cap;
    jsize len;
    jobject* objs;
    jlong* longs;
    char name[96];
};

static char exc_class[96], exc_msg[512];
static int pending;

static jobject mk(int kind) {
    jobject o = (jobject)calloc(1, sizeof(struct _jobject));
    o->kind = kind;
    return o;
}
static jclass f_find_class(JNIEnv* env, const char* name) {
    (void)env;
    jobject c = mk(K_CLASS);
    snprintf(c->name, sizeof c->name, "%s", name);
    return c;
}
static jint f_throw_new(JNIEnv* env, jclass cls, const char* msg) {
    (void)env;
    snprintf(exc_class, sizeof exc_class, "%s", cls->name);
    snprintf(exc_msg, sizeof exc_msg, "%s", msg);
    pending = 1;
    return 0;
}
static jboolean f_exception_check(JNIEnv* env) {
    (void)env;
    return (jboolean)pending;
}
static jsize f_array_length(JNIEnv* env, jarray a) {
    (void)env;
    return a->len;
}
static void f_set_obj(JNIEnv* env, jobjectArray a, jsize i, jobject v) {
    (void)env;
    a->objs[i] = v;
}
static jlong* f_get_longs(JNIEnv* env, jlongArray a, jboolean* copy) {
    (void)env;
    if (copy) *copy = JNI_FALSE;
    return a->longs;
}
static void f_release_longs(JNIEnv* env, jlongArray a, jlong* e, jint mode) {
    (void)env;
    (void)a;
    (void)e;
    (void)mode;
}
static void f_set_long_region(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* b) {
    (void)env;
    memcpy(a->longs + s, b, sizeof(jlong) * (size_t)n);
}
static jobject f_new_direct(JNIEnv* env, void* p, jlong cap) {
    (void)env;
    jobject o = mk(K_DIRECT);
    o->addr = p;
    o->cap = cap;
    return o;
}
static void* f_direct_addr(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->addr : NULL;
}
static jlong f_direct_cap(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->cap : -1;
}

static jlongArray f_new_longs(JNIEnv* env, jsize len) {
    (void)env;
    jobject o = mk(K_LONGARR);
    o->len = len;
    o->longs = (jlong*)calloc((size_t)(len > 0 ? len : 1), sizeof(jlong));
    return o;
}

static const struct JNINativeInterface_ table = {
    f_find_class,  f_throw_new,     f_exception_check, f_array_length, f_set_obj, f_get_longs,
    f_release_longs, f_set_long_region, f_new_direct, f_direct_addr,   f_direct_cap, f_new_longs,
};
static JNIEnv envp = &table;
static JNIEnv* env = &envp;

#define FN(name) Java_org_apache_flink_table_runtime_operators_window_gpu_FlinkGpu_##name
jlong FN(open)(JNIEnv*, jclass, jobject, jlongArray, jlongArray);
void FN(addBatch)(JNIEnv*, jclass, jlong, jobject, jobject, jobject, jobject, jint);
jlong FN(advanceProgress)(JNIEnv*, jclass, jlong, jlong, jobjectArray);
void FN(advanceProgressAsync)(JNIEnv*, jclass, jlong, jlong);
jlong FN(collectFired)(JNIEnv*, jclass, jlong, jobjectArray);
jlong FN(flushPartials)(JNIEnv*, jclass, jlong, jobjectArray);
void FN(snapshotStateAsync)(JNIEnv*, jclass, jlong);
jlong FN(snapshotStateWait)(JNIEnv*, jclass, jlong, jobjectArray, jlongArray);
jlong FN(lateDropped)(JNIEnv*, jclass, jlong);
void FN(close)(JNIEnv*, jclass, jlong);
void FN(hostRegister)(JNIEnv*, jclass, jint, jobject);
void FN(commUniqueId)(JNIEnv*, jclass, jobject);
jlong FN(commOpen)(JNIEnv*, jclass, jint, jint, jint, jobject);
jlong FN(commExchangeFired)(JNIEnv*, jclass, jlong, jlong, jint, jint, jlong, jlong);
jlong FN(commBytesSent)(JNIEnv*, jclass, jlong);
void FN(commClose)(JNIEnv*, jclass, jlong);
jlongArray FN(snapshotSlices)(JNIEnv*, jclass, jlong);
void FN(commRoundBegin)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jlong, jlong);
void FN(commRoundExchange)(JNIEnv*, jclass, jlong, jlongArray);
void FN(commRoundEnd)(JNIEnv*, jclass, jlong, jlong);

static jobject direct(void* p, jlong cap) { return f_new_direct(env, p, cap); }
static jobject objarr(jsize n) {
    jobject a = mk(K_OBJARR);
    a->len = n;
    a->objs = (jobject*)calloc((size_t)n, sizeof(jobject));
    return a;
}
static jobject longarr(jsize n) {
    jobject a = mk(K_LONGARR);
    a->len = n;
    a->longs = (jlong*)calloc((size_t)n, sizeof(jlong));
    return a;
}

static int failures;

static void expect_exc(const char* what, const char* cls, const char* msg) {
    if (!pending || strcmp(exc_class, cls) != 0 || (msg && strstr(exc_msg, msg) == NULL)) {
        printf("FAIL %s: pending %d class '%s' message '%s' (expected %s '%s')\n", what, pending, exc_class, exc_msg,
               cls, msg ? msg : "*");
        failures++;
    }
    pending = 0;
}

static fg_config config(int kind, long long size, long long slide, long long offset, int cs) {
    fg_config c;
    memset(&c, 0, sizeof c);
    c.window_kind = kind;
    c.size_ms = size;
    c.slide_ms = slide;
    c.offset_ms = offset;
    c.val_type = FG_VAL_F64;
    c.num_aggs = cs ? 3 : 2;
    c.aggs[0] = cs ? FG_AGG_COUNT_STAR : FG_AGG_SUM;
    c.aggs[1] = FG_AGG_SUM;
    c.aggs[2] = FG_AGG_AVG;
    c.max_parallelism = 128;
    c.key_group_end = 127;
    c.expected_keys = 16;
    c.buffer_records = 1 << 16;
    return c;
}

static int errors_mode(void) {
    char line[1024];
    int cases = 0;
    while (fgets(line, sizeof line, stdin)) {
        int kind, cs, off = 0;
        long long size, slide, offset;
        if (sscanf(line, "spec %d %lld %lld %lld %d %n", &kind, &size, &slide, &offset, &cs, &off) < 5) continue;
        char* msg = line + off;
        msg[strcspn(msg, "\n")] = 0;
        fg_config c = config(kind, size, slide, offset, cs);
        jlong h = FN(open)(env, NULL, direct(&c, sizeof c), NULL, NULL);
        if (h) FN(close)(env, NULL, h);
        expect_exc("window spec", "java/lang/IllegalArgumentException", msg);
        if (strcmp(exc_msg, msg) != 0 && failures == 0) {
            printf("FAIL message '%s' expected '%s'\n", exc_msg, msg);
            failures++;
        }
        cases++;
    }
    /* a heap ByteBuffer (no direct address) */
    jobject heap = mk(K_HEAP);
    FN(open)(env, NULL, heap, NULL, NULL);
    expect_exc("heap config buffer", "java/lang/IllegalArgumentException", "direct ByteBuffers only");
    FN(addBatch)(env, NULL, 0, heap, heap, NULL, NULL, 4);   /* throws before the handle is used */
    expect_exc("heap batch buffer", "java/lang/IllegalArgumentException", "direct ByteBuffers only");
    FN(hostRegister)(env, NULL, 0, heap);
    expect_exc("heap segment", "java/lang/IllegalArgumentException", "direct ByteBuffers only");
    /* zone rules: n transitions need n instants and n + 1 offsets */
    fg_config z = config(FG_TUMBLE, 1000, 0, 0, 1);
    z.n_tz_transitions = 2;
    FN(open)(env, NULL, direct(&z, sizeof z), longarr(2), longarr(2));
    expect_exc("zone rules", "java/lang/IllegalArgumentException", "zone rules need");
    cases += 4;
    /* a valid spec: a handle on a GPU host, RuntimeException (FG_EDEVICE) without one */
    fg_config v = config(FG_TUMBLE, 1000, 0, 0, 1);
    jlong h = FN(open)(env, NULL, direct(&v, sizeof v), NULL, NULL);
    if (h) {
        FN(close)(env, NULL, h);
    } else {
        expect_exc("valid spec without a device", "java/lang/RuntimeException", "no HIP device");
    }
    cases++;
    printf("%d cases, %d failures\n", cases, failures);
    return failures ? 1 : 0;
}

/* the sums of a fired column set: rows, COUNT(*) total, SUM total (host reads of every column) */
static void totals(const char* tag, jobjectArray cols, jlong n, int num_aggs) {
    const int64_t* key = (const int64_t*)cols->objs[0]->addr;
    const int64_t* we = (const int64_t*)cols->objs[2]->addr;
    const int64_t* a0 = (const int64_t*)cols->objs[3]->addr;
    const double* a1 = (const double*)cols->objs[4]->addr;
    long long cnt = 0, keys = 0, ends = 0;
    double sum = 0;
    for (jlong i = 0; i < n; i++) {
        cnt += a0[i];
        sum += a1[i];
        keys += key[i];
        ends += we[i];
    }
    (void)num_aggs;
    printf("%s rows %lld count %lld sum %.1f keysum %lld endsum %lld\n", tag, (long long)n, cnt, sum, keys, ends);
}

static int gpu_mode(void) {
    enum { N = 1000 };
    static int64_t key[N], rt[N];
    static double val[N];
    for (int i = 0; i < N; i++) {
        key[i] = i % 10;
        rt[i] = 5LL * i;
        val[i] = 1.0 + i % 3;
    }
    fg_config c = config(FG_TUMBLE, 1000, 0, 0, 1);
    jlong h = FN(open)(env, NULL, direct(&c, sizeof c), NULL, NULL);
    if (!h) {
        printf("FAIL open: %s %s\n", exc_class, exc_msg);
        return 1;
    }
    FN(addBatch)(env, NULL, h, direct(key, sizeof key), direct(rt, sizeof rt), direct(val, sizeof val), NULL, N);
    FN(advanceProgressAsync)(env, NULL, h, 2999);
    jobjectArray cols = objarr(10);
    jlong n = FN(collectFired)(env, NULL, h, cols);
    totals("async", cols, n, 3);
    /* the state as of here (windows ending 4000 and 5000), collected after the next advance fired them */
    FN(snapshotStateAsync)(env, NULL, h);
    n = FN(advanceProgress)(env, NULL, h, 10000, cols);
    totals("sync", cols, n, 3);
    {
        jobjectArray sc = objarr(7);
        jlongArray swm = longarr(1);
        jlong sn = FN(snapshotStateWait)(env, NULL, h, sc, swm);
        const int64_t* cs = (const int64_t*)sc->objs[2]->addr;
        long long t = 0;
        for (jlong i = 0; i < sn; i++) t += cs[i];
        printf("snapshot entries %lld cnt_star %lld wm %lld\n", (long long)sn, t, (long long)swm->longs[0]);
        /* the image's slices: [n, ends, first rows, rows, changed] */
        jlongArray sl = FN(snapshotSlices)(env, NULL, h);
        const jlong* v = sl->longs;
        const jlong ns = v[0];
        long long rows = 0, changed = 0;
        for (jlong i = 0; i < ns; i++) {
            rows += v[1 + 2 * ns + i];
            changed += v[1 + 3 * ns + i];
        }
        printf("slices %lld first_end %lld rows %lld changed %lld\n", (long long)ns, (long long)(ns ? v[1] : 0), rows,
               changed);
    }
    printf("late %lld\n", (long long)FN(lateDropped)(env, NULL, h));
    FN(close)(env, NULL, h);
    /* the local phase: partial rows of every buffered slice */
    c.flags = FG_FLAG_LOCAL_PARTIALS;
    h = FN(open)(env, NULL, direct(&c, sizeof c), NULL, NULL);
    FN(addBatch)(env, NULL, h, direct(key, sizeof key), direct(rt, sizeof rt), direct(val, sizeof val), NULL, N);
    n = FN(flushPartials)(env, NULL, h, cols);
    {   /* partial columns: agg[0] COUNT(*), agg[1] COUNT(v), agg[2] SUM bits */
        const int64_t* cs = (const int64_t*)cols->objs[3]->addr;
        const int64_t* cv = (const int64_t*)cols->objs[4]->addr;
        const double* s = (const double*)cols->objs[5]->addr;
        long long a = 0, b = 0;
        double t = 0;
        for (jlong i = 0; i < n; i++) {
            a += cs[i];
            b += cv[i];
            t += s[i];
        }
        printf("partials rows %lld cnt_star %lld cnt_val %lld sum %.1f\n", (long long)n, a, b, t);
    }
    FN(close)(env, NULL, h);
    {   /* the two-phase edge over RCCL at world size 1: local partials -> exchange -> global */
        static uint8_t id[FG_COMM_ID_BYTES];
        FN(commUniqueId)(env, NULL, direct(id, sizeof id));
        jlong comm = FN(commOpen)(env, NULL, 0, 1, 0, direct(id, sizeof id));
        if (!comm) {
            printf("FAIL commOpen: %s %s\n", exc_class, exc_msg);
            return 1;
        }
        fg_config lc = config(FG_TUMBLE, 1000, 0, 0, 1);
        lc.flags = FG_FLAG_LOCAL_PARTIALS;
        fg_config gc = config(FG_TUMBLE, 1000, 0, 0, 1);
        jlong loc = FN(open)(env, NULL, direct(&lc, sizeof lc), NULL, NULL);
        jlong glob = FN(open)(env, NULL, direct(&gc, sizeof gc), NULL, NULL);
        FN(addBatch)(env, NULL, loc, direct(key, sizeof key), direct(rt, sizeof rt), direct(val, sizeof val), NULL, N);
        FN(advanceProgressAsync)(env, NULL, loc, 2999);
        jlong mw = FN(commExchangeFired)(env, NULL, comm, loc, FG_KEYHASH_BINARYROW_BIGINT, 128, 2999, glob);
        printf("comm_wm %lld sent %lld\n", (long long)mw, (long long)FN(commBytesSent)(env, NULL, comm));
        n = FN(advanceProgress)(env, NULL, glob, mw, cols);
        totals("comm", cols, n, 3);
        /* the same edge as a round (commRoundBegin / Exchange / End: the fused operator's edge
         * thread): the records of the windows ending 4000 .. 5000 at the final watermark */
        FN(advanceProgressAsync)(env, NULL, loc, 10000);
        FN(commRoundBegin)(env, NULL, comm, loc, 0 /* ROUND_FIRED */, FG_KEYHASH_BINARYROW_BIGINT, 128, 10000, 7);
        jlongArray ro = longarr(5);
        FN(commRoundExchange)(env, NULL, comm, ro);
        FN(commRoundEnd)(env, NULL, comm, glob);
        printf("round_wm %lld epoch %lld sent %lld received %lld\n", (long long)ro->longs[0], (long long)ro->longs[1],
               (long long)ro->longs[2], (long long)ro->longs[3]);
        n = FN(advanceProgress)(env, NULL, glob, ro->longs[0], cols);
        totals("round", cols, n, 3);
        /* an idle round (nothing to send; local may be 0) */
        FN(commRoundBegin)(env, NULL, comm, 0, 2 /* ROUND_IDLE */, FG_KEYHASH_BINARYROW_BIGINT, 128, 10001, 8);
        FN(commRoundExchange)(env, NULL, comm, ro);
        FN(commRoundEnd)(env, NULL, comm, glob);
        printf("idle_wm %lld epoch %lld received %lld\n", (long long)ro->longs[0], (long long)ro->longs[1],
               (long long)ro->longs[3]);
        FN(close)(env, NULL, loc);
        FN(close)(env, NULL, glob);
        FN(commClose)(env, NULL, comm);
    }
    if (pending) {
        printf("FAIL pending exception %s: %s\n", exc_class, exc_msg);
        return 1;
    }
    printf("gpu done\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) return gpu_mode();
    return errors_mode();
}

/* Host-logic driver of libflinkgpu_asan.so (flink_amd/Makefile `asan`: fg_engine.cpp and
 * fg_keydict.hip host code under AddressSanitizer + UndefinedBehaviorSanitizer). Test
 * infrastructure only (tests/test_asan.py). Runs without a GPU: every C-ABI path that must not
 * touch a device -- window-spec validation with the reference's messages, argument checks, the
 * BinaryRowData hash, error reporting on NULL handles -- and fg_open of a valid spec, which
 * fails with FG_EDEVICE when no device is present.
 *
 * stdin lines:
 *   spec <kind> <size> <slide> <offset> <mode> <count_star 0/1> <expected rc> <expected message or ->
 *   hash <hex row bytes> <expected int32>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flinkgpu.h"

static int failures = 0;

static void spec_case(int kind, long long size, long long slide, long long offset, int mode, int cs, int exp_rc,
                      const char* msg) {
    fg_config c;
    memset(&c, 0, sizeof c);
    c.mode = mode;
    c.window_kind = kind;
    c.size_ms = size;
    c.slide_ms = slide;
    c.offset_ms = offset;
    c.val_type = FG_VAL_F64;
    c.num_aggs = cs ? 2 : 1;   /* (no COUNT(*): SliceAssigners' hopping count-star check) */
    c.aggs[0] = cs ? FG_AGG_COUNT_STAR : FG_AGG_SUM;
    c.aggs[1] = FG_AGG_SUM;
    c.max_parallelism = 128;
    c.key_group_end = 127;
    c.expected_keys = 1000;
    c.buffer_records = 1 << 16;
    fg_handle* h = NULL;
    const int rc = fg_open(&c, &h);
    const char* err = fg_last_error(NULL);
    if (exp_rc == FG_OK) {   /* a valid spec: FG_OK on a GPU host, FG_EDEVICE without one */
        if (rc != FG_OK && rc != FG_EDEVICE) {
            printf("FAIL spec %d %lld: rc %d (%s)\n", kind, size, rc, err);
            failures++;
        }
    } else if (rc != exp_rc || (strcmp(msg, "-") != 0 && strcmp(err, msg) != 0)) {
        printf("FAIL spec %d %lld %lld %lld: rc %d expected %d, message '%s' expected '%s'\n", kind, size, slide, offset,
               rc, exp_rc, err, msg);
        failures++;
    }
    if (h) fg_close(h);
}

static int hexval(char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

int main(void) {
    char line[4096];
    int cases = 0;
    if (fg_abi_version() != FG_ABI_VERSION) {
        printf("FAIL abi version\n");
        failures++;
    }
    fg_close(NULL);   /* NULL handles are tolerated */
    if (fg_add_batch(NULL, NULL) != FG_EINVAL || fg_flush(NULL) != FG_EINVAL || fg_open(NULL, NULL) != FG_EINVAL) {
        printf("FAIL NULL-handle checks\n");
        failures++;
    }
    while (fgets(line, sizeof line, stdin)) {
        char kw[16];
        if (sscanf(line, "%15s", kw) != 1) continue;
        if (strcmp(kw, "spec") == 0) {
            int kind, mode, cs, exp_rc, off = 0;
            long long size, slide, offset;
            if (sscanf(line, "spec %d %lld %lld %lld %d %d %d %n", &kind, &size, &slide, &offset, &mode, &cs, &exp_rc, &off) < 7)
                continue;
            char* msg = line + off;
            msg[strcspn(msg, "\n")] = 0;
            spec_case(kind, size, slide, offset, mode, cs, exp_rc, msg);
            cases++;
        } else if (strcmp(kw, "hash") == 0) {
            char hex[3000];
            int expected;
            if (sscanf(line, "hash %2999s %d", hex, &expected) != 2) continue;
            const size_t n = strlen(hex) / 2;
            unsigned char* row = (unsigned char*)malloc(n);
            for (size_t i = 0; i < n; i++) row[i] = (unsigned char)(hexval(hex[2 * i]) << 4 | hexval(hex[2 * i + 1]));
            const int got = fg_binaryrow_hash(row, (int)n);
            if (got != expected) {
                printf("FAIL hash of %zu bytes: %d expected %d\n", n, got, expected);
                failures++;
            }
            free(row);
            cases++;
        }
    }
    printf("%d cases, %d failures\n", cases, failures);
    return failures ? 1 : 0;
}

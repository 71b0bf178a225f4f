/*
 * thread_fuzz.c - the combine dispatcher (libucg_builtin.so) and its device
 * context shared by several host threads, as UCG shares them between the
 * progress thread and the UCS async timer thread that resends and drains
 * stashed fragments (builtin/builtin.c:284-294): one thread
 * runs staged REDUCE steps fragment by fragment, three threads run
 * whole-buffer combines on host (pageable or pinned) and device-resident
 * buffers, all on ONE combine object. Every result is checked bit for bit
 * against the oracle (test infrastructure) applying reduce_cb_f's
 * restatement in the same order.
 *
 *   thread_fuzz [iterations=60] [seed]
 *
 * Prints one JSON line; exit 3 on a mismatch.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ucg_builtin_combine.h"
#include "combine_ref.h"

/* opaque MPI handles: op + 1 and dtype + 1 */
#define OPH(o) ((void*)(uintptr_t)((o) + 1))
#define DTH(d) ((void*)(uintptr_t)((d) + 1))
#define OPI(h) ((int)(uintptr_t)(h) - 1)
#define DTI(h) ((int)(uintptr_t)(h) - 1)

static int reduce_cb(void *op, char *src, char *dst, unsigned count, void *dt)
{
    return ucg_oracle_reduce(OPI(op), DTI(dt), src, dst, count);
}
static int is_sum(void *op) { return OPI(op) == ORA_SUM; }
static int no(void *op) { (void)op; return 0; }
static int yes(void *op) { (void)op; return 1; }
static int convert(void *dt, uintptr_t *u)
{
    *u = (uintptr_t)ucg_oracle_dtype_size(DTI(dt)) << 3;   /* contiguous */
    return 0;
}
static int is_float_dt(int d) { return d >= 8; }
static int is_int(void *dt, int *s) { *s = DTI(dt) % 2 == 0; return !is_float_dt(DTI(dt)); }
static int is_fp(void *dt) { return is_float_dt(DTI(dt)); }
static int op_cls(void *op) { return OPI(op); }
static int dt_cls(void *dt) { return DTI(dt); }

static ucg_builtin_combine_t *g_cmb;
static int g_iters;
static volatile int g_fail;
static uint64_t g_seed;

static uint64_t rnd(uint64_t *s)
{
    *s += 0x9E3779B97F4A7C15ull;
    return ucg_oracle_splitmix64(*s);
}

static void pick(uint64_t *s, int *dt, int *op)
{
    do {
        *dt = (int)(rnd(s) % UCG_DEV_DT_LAST);
        *op = (int)(rnd(s) % UCG_DEV_OP_LAST);
    } while (!ucg_oracle_is_supported(*dt, *op));
}

/* staged steps: begin, every fragment borrowed for the call only, end */
static void *stage_thread(void *arg)
{
    uint64_t s = g_seed ^ 0x51A6Eull;
    int it;
    (void)arg;
    for (it = 0; it < g_iters && !g_fail; it++) {
        int dt, op;
        pick(&s, &dt, &op);
        const size_t sz = ucg_oracle_dtype_size(dt);
        const size_t count = 1 + rnd(&s) % (120000 / sz);
        const size_t bytes = count * sz, frag = sz * (1 + rnd(&s) % (9000 / sz));
        char *acc = malloc(bytes), *want = malloc(bytes), *src = malloc(bytes);
        size_t off;
        ucg_oracle_fill(dt, ORA_DIST_ROUND, s, src, count);
        ucg_oracle_fill(dt, ORA_DIST_ROUND, s + 1, want, count);
        memcpy(acc, want, bytes);
        if (ucg_builtin_combine_step_begin(g_cmb, OPH(op), DTH(dt), acc, bytes) != UCS_OK) {
            fprintf(stderr, "step_begin failed\n");
            g_fail = 1;
            break;
        }
        for (off = 0; off < bytes; off += frag) {
            const size_t n = bytes - off < frag ? bytes - off : frag;
            char *am = malloc(n);
            memcpy(am, src + off, n);
            if (ucg_builtin_combine_fragment(g_cmb, off, am, n) != UCS_OK) {
                fprintf(stderr, "fragment failed\n");
                g_fail = 1;
            }
            memset(am, 0x5A, n);
            free(am);
            ucg_oracle_reduce(op, dt, src + off, want + off, n / sz);
        }
        if (ucg_builtin_combine_step_end(g_cmb) != UCS_OK || memcmp(acc, want, bytes)) {
            fprintf(stderr, "staged step %d MISMATCH dt=%d op=%d count=%zu frag=%zu\n", it,
                    dt, op, count, frag);
            g_fail = 3;
        }
        free(acc);
        free(want);
        free(src);
    }
    return NULL;
}

/* whole-buffer combines: kind 0 pageable, 1 pinned, 2 device-resident dst */
static void *whole_thread(void *arg)
{
    const int kind = (int)(uintptr_t)arg;
    uint64_t s = g_seed ^ (0xB0B0ull * (kind + 1));
    ucg_builtin_dev_ctx_t *dev = ucg_builtin_combine_dev_ctx(g_cmb);
    int it;
    for (it = 0; it < 2 * g_iters && !g_fail; it++) {
        int dt, op;
        pick(&s, &dt, &op);
        const size_t sz = ucg_oracle_dtype_size(dt);
        const size_t count = 1 + rnd(&s) % (200000 / sz);
        const size_t bytes = count * sz;
        char *src = malloc(bytes), *want = malloc(bytes), *got = malloc(bytes);
        char *dst = kind == 0 ? malloc(bytes) : kind == 1 ? ucg_builtin_dev_host_alloc(bytes)
                                                          : ucg_builtin_dev_malloc(dev, bytes);
        ucg_oracle_fill(dt, ORA_DIST_ROUND, s, src, count);
        ucg_oracle_fill(dt, ORA_DIST_ROUND, s + 7, want, count);
        if (kind == 2) {
            ucg_builtin_dev_memcpy(dev, dst, want, bytes);
        } else {
            memcpy(dst, want, bytes);
        }
        ucg_oracle_reduce(op, dt, src, want, count);
        if (ucg_builtin_combine_reduce(g_cmb, OPH(op), src, dst, (int)count, DTH(dt)) != UCS_OK) {
            fprintf(stderr, "combine_reduce failed\n");
            g_fail = 1;
        }
        if (kind == 2) {
            ucg_builtin_dev_memcpy(dev, got, dst, bytes);
        } else {
            memcpy(got, dst, bytes);
        }
        if (memcmp(got, want, bytes)) {
            fprintf(stderr, "whole-buffer (kind %d) %d MISMATCH dt=%d op=%d count=%zu\n", kind,
                    it, dt, op, count);
            g_fail = 3;
        }
        if (kind == 0) {
            free(dst);
        } else if (kind == 1) {
            ucg_builtin_dev_host_free(dst);
        } else {
            ucg_builtin_dev_free(dev, dst);
        }
        free(src);
        free(want);
        free(got);
    }
    return NULL;
}

int main(int argc, char **argv)
{
    ucg_builtin_reduce_params_t rp = {reduce_cb, is_sum, no, yes, convert, is_int, is_fp};
    /* force: host buffers of any size staged on the GPU; small slots and a
     * shallow ring so steps and whole-buffer calls share and reuse slots */
    ucg_builtin_combine_config_t cfg = {2, 0, 4096, 3, -1, 0, 0, NULL};
    pthread_t th[4];
    uint64_t st[6];
    int i;
    g_iters = argc > 1 ? atoi(argv[1]) : 60;
    g_seed  = argc > 2 ? strtoull(argv[2], NULL, 0) : 0x7E4Dull;
    if (ucg_builtin_combine_create(&rp, &cfg, &g_cmb) != UCS_OK ||
        !ucg_builtin_combine_has_device(g_cmb)) {
        fprintf(stderr, "no device combine\n");
        return 1;
    }
    ucg_builtin_combine_set_classifier(g_cmb, op_cls, dt_cls);
    pthread_create(&th[0], NULL, stage_thread, NULL);
    for (i = 0; i < 3; i++) {
        pthread_create(&th[1 + i], NULL, whole_thread, (void*)(uintptr_t)i);
    }
    for (i = 0; i < 4; i++) {
        pthread_join(th[i], NULL);
    }
    ucg_builtin_combine_stats(g_cmb, st);
    printf("{\"harness\": \"thread_fuzz\", \"threads\": 4, \"staged_steps\": %d, "
           "\"whole_buffer_calls\": %d, \"device_calls\": %llu, \"host_calls\": %llu, "
           "\"steps_on_device\": %llu, \"bit_exact\": %s}\n", g_iters, 6 * g_iters,
           (unsigned long long)st[2], (unsigned long long)st[0],
           (unsigned long long)st[4], g_fail ? "false" : "true");
    ucg_builtin_combine_destroy(g_cmb);
    return g_fail ? (g_fail == 3 ? 3 : 1) : 0;
}

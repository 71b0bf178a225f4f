/*
 * multi_group_timers.c - several groups on ONE transport object, each with
 * its resend timer thread, ops of all of them in flight at once.
 *
 *   RANK=r WORLD_SIZE=n multi_group_timers <shm-name> [groups = 3] [iters = 40]
 *
 * The reference's groups of one worker share the worker's async context:
 * UCS_ASYNC_BLOCK is one lock for the transport, the group table and the
 * unexpected-message list they all reach (builtin/builtin.c:133-219, 284-294,
 * 408-413). Here every group's timer progresses the shared transport and may
 * deliver another group's messages, so the engine's lock is the interface's.
 * Every iteration starts an allreduce on every group (a 2-cell ring: the
 * sends stop at UCS_ERR_NO_RESOURCE and the timers resend), then waits for
 * them in reverse order; the sums are exact. Built plain and under
 * ThreadSanitizer (tests/c/Makefile, test_engine_thread_sanitizer).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ucg_builtin_ops.h"

#define MAXG 8

static int sum_f32(void *op, char *src, char *dst, unsigned count, void *dt)
{
    unsigned i;
    (void)op;
    (void)dt;
    for (i = 0; i < count; i++) {
        ((float*)dst)[i] = ((float*)src)[i] + ((float*)dst)[i];
    }
    return 0;
}

static int yes(void *op) { (void)op; return 1; }
static int no(void *op) { (void)op; return 0; }
static int convert(void *dt, uintptr_t *u) { (void)dt; *u = 4u << 3; return 0; }
static int is_int(void *dt, int *s) { (void)dt; *s = 0; return 0; }
static int is_fp(void *dt) { (void)dt; return 1; }

int main(int argc, char **argv)
{
    const unsigned rank  = (unsigned)atoi(getenv("RANK"));
    const unsigned world = (unsigned)atoi(getenv("WORLD_SIZE"));
    const unsigned ng    = argc > 2 ? (unsigned)atoi(argv[2]) : 3;
    const int iters      = argc > 3 ? atoi(argv[3]) : 40;
    const int count      = 2048;                    /* 33 fragments of 248 B */
    ucg_builtin_reduce_params_t rp = {sum_f32, yes, no, yes, convert, is_int, is_fp};
    ucg_builtin_combine_config_t cfg;
    ucg_builtin_combine_t *cmb[MAXG];
    ucg_builtin_lgroup_t *g[MAXG];
    ucg_builtin_lcoll_t *c[MAXG];
    float *in[MAXG], *out[MAXG];
    ucg_builtin_shm_iface_t *iface;
    ucs_status_t st;
    unsigned k;
    int it, i, ok = 1;

    if (argc < 2 || ng == 0 || ng > MAXG) {
        fprintf(stderr, "usage: multi_group_timers <shm-name> [groups <= %d] [iters]\n", MAXG);
        return 2;
    }
    ucg_builtin_combine_config_read(&cfg);
    cfg.dev_enable = 0;
    if (ucg_builtin_shm_iface_open(argv[1], world, rank, 256, 2, &iface) != UCS_OK) {
        fprintf(stderr, "rank %u: open failed\n", rank);
        return 1;
    }
    for (k = 0; k < ng; k++) {
        in[k]  = malloc(count * sizeof(float));
        out[k] = malloc(count * sizeof(float));
        for (i = 0; i < count; i++) {
            in[k][i] = (float)((int)(rank * 131 + k * 17 + i) % 512);
        }
        if (ucg_builtin_combine_create(&rp, &cfg, &cmb[k]) != UCS_OK ||
            ucg_builtin_lgroup_create(iface, (uint16_t)(k + 1), world, rank, cmb[k], &g[k]) !=
                UCS_OK ||
            ucg_builtin_lcoll_allreduce(g[k], in[k], out[k], count, (void*)1, (void*)1,
                                        &c[k]) != UCS_OK ||
            ucg_builtin_lgroup_set_async_timer(g[k], 0.001) != UCS_OK) {
            fprintf(stderr, "rank %u: group %u set-up failed\n", rank, k + 1);
            return 1;
        }
    }
    if (ucg_builtin_shm_barrier(iface) != UCS_OK) {
        return 1;
    }
    for (it = 0; it < iters && ok; it++) {
        for (k = 0; k < ng; k++) {
            st = ucg_builtin_lcoll_start(c[k]);
            if (st != UCS_OK && st != UCS_INPROGRESS) {
                fprintf(stderr, "rank %u: start %u: %d\n", rank, k, st);
                ok = 0;
            }
        }
        for (k = ng; k-- > 0 && ok;) {
            if ((st = ucg_builtin_lcoll_wait(c[k])) != UCS_OK) {
                fprintf(stderr, "rank %u: iteration %d group %u: status %d\n", rank, it, k + 1,
                        st);
                ok = 0;
                break;
            }
            for (i = 0; i < count; i++) {
                float want = 0.0f;
                unsigned r;
                for (r = 0; r < world; r++) {
                    want += (float)((int)(r * 131 + k * 17 + i) % 512);
                }
                if (out[k][i] != want) {
                    fprintf(stderr, "rank %u: iteration %d group %u element %d: %g != %g\n",
                            rank, it, k + 1, i, out[k][i], want);
                    ok = 0;
                    break;
                }
            }
        }
    }
    if (ucg_builtin_shm_barrier(iface) != UCS_OK) {
        ok = 0;
    }
    for (k = 0; k < ng; k++) {
        ucg_builtin_lcoll_destroy(c[k]);
        ucg_builtin_lgroup_destroy(g[k]);
        ucg_builtin_combine_destroy(cmb[k]);
        free(in[k]);
        free(out[k]);
    }
    if (ucg_builtin_shm_iface_close(iface) != UCS_OK) {
        ok = 0;
    }
    printf("rank %u: %s\n", rank, ok ? "ok" : "FAILED");
    return ok ? 0 : 1;
}

/*
 * async_resend.c - the resend timer of the group's async context (SURVEY.md
 * 8a row a15; builtin/builtin.c:260-294, 408-413) on two processes.
 *
 *   RANK=r WORLD_SIZE=2 async_resend <shm-name> [host|staged|device]
 *
 * The transport has 2 cells per ring, so an allreduce of 133 fragments stops
 * at UCS_ERR_NO_RESOURCE at once on both members. Phases (shm barriers):
 *   1. member 1 starts and stops sending; member 0 starts, stops, and
 *      progresses: member 1's first fragments arrive while member 0's step
 *      has not finished sending, so they are stashed (builtin.c:207-216);
 *   2. member 0 stops calling into the engine (sleeps) while member 1
 *      progresses: only member 0's resend timer thread sends its fragments,
 *      and once they are all out that thread drains the stash - the combine
 *      runs on the async thread, as in the reference;
 *   3. both wait for completion: bit-exact sums on both members.
 * Modes (the combine's HIP calls on the timer thread):
 *   host    host buffers, every combine on the host (reduce_cb_f)
 *   staged  host buffers, every step staged on the GPU (UCX_BUILTIN_DEV_COMBINE
 *           =force): the timer thread's combines are device launches
 *           (ucg_builtin_dev_combine / stage_end)
 *   device  device buffers: remote-key steps. Member 1 also runs a timer, so
 *           its READY reaches member 0 while member 0's own messages are
 *           still stuck; member 0's fold waits for its sends (rma_receive)
 *           and runs on member 0's timer thread once they go out.
 * Member 0 prints the timer's resend and combine counts and the combine
 * layer's host / device call counts.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "ucg_builtin_ops.h"
#include "ucg_builtin_dev.h"

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
/* the device enums of the only (op, dtype) this "MPI library" knows */
static int classify_op(void *op) { (void)op; return UCG_DEV_OP_SUM; }
static int classify_dt(void *dt) { (void)dt; return UCG_DEV_DT_FLOAT32; }

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int run(char **argv, const char *mode);

int main(int argc, char **argv)
{
    return run(argv, argc > 2 ? argv[2] : "host");
}

static int run(char **argv, const char *mode)
{
    const unsigned rank = (unsigned)atoi(getenv("RANK"));
    const int count = 8192 * 4 / 4;                /* 32 KiB: 133 fragments of 248 B */
    const int staged = strcmp(mode, "staged") == 0, device = strcmp(mode, "device") == 0;
    ucg_builtin_reduce_params_t rp = {sum_f32, yes, no, yes, convert, is_int, is_fp};
    ucg_builtin_combine_config_t cfg;
    ucg_builtin_combine_t *cmb;
    ucg_builtin_shm_iface_t *iface;
    ucg_builtin_lgroup_t *g;
    ucg_builtin_lcoll_t *c;
    ucg_builtin_dev_ctx_t *dctx = NULL;
    float *in = malloc(count * sizeof(float)), *out = calloc(count, sizeof(float));
    void *sbuf = in, *rbuf = out;
    uint64_t st4[4], as[2], cs[6], sent_before;
    ucs_status_t st;
    int i, ok = 1;

    ucg_builtin_combine_config_read(&cfg);
    cfg.dev_enable = staged ? 2 : device ? 1 : 0;
    if (staged) {
        cfg.dev_min_bytes = 0;                     /* every step on the GPU */
    }
    for (i = 0; i < count; i++) {
        in[i] = (float)((int)(rank * 1000 + i) % 4096 - 2048);
    }
    if (ucg_builtin_combine_create(&rp, &cfg, &cmb) != UCS_OK) {
        fprintf(stderr, "rank %u: combine set-up failed\n", rank);
        return 1;
    }
    if (staged || device) {
        ucg_builtin_combine_set_classifier(cmb, classify_op, classify_dt);
        if (!ucg_builtin_combine_has_device(cmb)) {
            fprintf(stderr, "rank %u: no device\n", rank);
            return 2;
        }
    }
    if (device) {
        ucg_builtin_dev_ctx_params_t dp;
        memset(&dp, 0, sizeof(dp));
        if (ucg_builtin_dev_ctx_create(&dp, &dctx) != UCS_OK ||
            (sbuf = ucg_builtin_dev_malloc(dctx, count * sizeof(float))) == NULL ||
            (rbuf = ucg_builtin_dev_malloc(dctx, count * sizeof(float))) == NULL ||
            ucg_builtin_dev_memcpy(dctx, sbuf, in, count * sizeof(float)) != UCS_OK ||
            ucg_builtin_dev_memcpy(dctx, rbuf, out, count * sizeof(float)) != UCS_OK) {
            fprintf(stderr, "rank %u: device buffers: %s\n", rank,
                    ucg_builtin_dev_last_error());
            return 1;
        }
    }
    if (ucg_builtin_shm_iface_open(argv[1], 2, rank, 256, 2, &iface) != UCS_OK ||
        ucg_builtin_lgroup_create(iface, 1, 2, rank, cmb, &g) != UCS_OK ||
        ucg_builtin_lcoll_allreduce(g, sbuf, rbuf, count, (void*)1, (void*)1, &c) != UCS_OK) {
        fprintf(stderr, "rank %u: set-up failed\n", rank);
        return 1;
    }
    if ((rank == 0 || device) && ucg_builtin_lgroup_set_async_timer(g, 0.005) != UCS_OK) {
        fprintf(stderr, "timer failed\n");
        return 1;
    }
    ucg_builtin_shm_barrier(iface);
    if (rank == 1) {
        st = ucg_builtin_lcoll_start(c);                 /* stops at the full ring */
        ucg_builtin_shm_barrier(iface);                  /* B1 */
        ucg_builtin_shm_barrier(iface);                  /* B2 */
        st = (st == UCS_INPROGRESS) ? ucg_builtin_lcoll_wait(c) : st;
    } else {
        double t0;
        ucg_builtin_shm_barrier(iface);                  /* B1 */
        st = ucg_builtin_lcoll_start(c);
        /* stash member 1's fragments (device: take in member 1's READY,
         * which member 1's timer sends once this member drained its ring) */
        t0 = now_s();
        for (i = 0; i < 1000 || (device && now_s() - t0 < 0.3); i++) {
            ucg_builtin_lgroup_progress(g);
        }
        ucg_builtin_lgroup_stats(g, st4);
        sent_before = st4[0];
        ucg_builtin_shm_barrier(iface);                  /* B2 */
        usleep(1500 * 1000);                             /* the timer thread works alone */
        ucg_builtin_lgroup_async_stats(g, as);
        ucg_builtin_lgroup_stats(g, st4);
        ucg_builtin_combine_stats(cmb, cs);
        printf("{\"mode\": \"%s\", \"sent_before_sleep\": %llu, \"sent_after_sleep\": %llu, "
               "\"stashed\": %llu, \"timer_resends\": %llu, \"timer_combines\": %llu, "
               "\"host_calls\": %llu, \"device_calls\": %llu, \"staged_steps\": %llu}\n",
               mode, (unsigned long long)sent_before, (unsigned long long)st4[0],
               (unsigned long long)st4[2], (unsigned long long)as[0],
               (unsigned long long)as[1], (unsigned long long)cs[0],
               (unsigned long long)cs[2], (unsigned long long)cs[4]);
        if (as[0] == 0 || as[1] == 0 || (!device && st4[0] != 133)) {
            fprintf(stderr, "rank 0: the timer thread did not resend and combine\n");
            ok = 0;
        }
        if ((staged && (cs[0] != 0 || cs[4] == 0)) || (device && cs[0] != 0)) {
            fprintf(stderr, "rank 0: a combine ran on the host\n");
            ok = 0;
        }
        st = (st == UCS_INPROGRESS) ? ucg_builtin_lcoll_wait(c) : st;
    }
    if (device && st == UCS_OK &&
        ucg_builtin_dev_memcpy(dctx, out, rbuf, count * sizeof(float)) != UCS_OK) {
        fprintf(stderr, "rank %u: download: %s\n", rank, ucg_builtin_dev_last_error());
        ok = 0;
    }
    for (i = 0; i < count && st == UCS_OK; i++) {
        const float want = (float)((int)i % 4096 - 2048) + (float)((int)(1000 + i) % 4096 - 2048);
        if (out[i] != want) {
            fprintf(stderr, "rank %u: element %d: %g != %g\n", rank, i, out[i], want);
            ok = 0;
            break;
        }
    }
    if (st != UCS_OK) {
        fprintf(stderr, "rank %u: status %d (%s)\n", rank, st,
                (staged || device) ? ucg_builtin_dev_last_error() : "");
        ok = 0;
    }
    ucg_builtin_shm_barrier(iface);
    ucg_builtin_lcoll_destroy(c);
    ucg_builtin_lgroup_destroy(g);
    ucg_builtin_shm_iface_close(iface);
    ucg_builtin_combine_destroy(cmb);
    if (dctx) {
        ucg_builtin_dev_free(dctx, sbuf);
        ucg_builtin_dev_free(dctx, rbuf);
        ucg_builtin_dev_ctx_destroy(dctx);
    }
    free(in);
    free(out);
    printf("rank %u: %s\n", rank, ok ? "ok" : "FAILED");
    return ok ? 0 : 1;
}

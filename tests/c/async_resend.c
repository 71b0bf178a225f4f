/*
 * async_resend.c - the resend timer of the group's async context (SURVEY.md
 * 8a row a15; builtin/builtin.c:260-294, 408-413) on two processes.
 *
 *   RANK=r WORLD_SIZE=2|4 async_resend <shm-name> [host|staged|device] [exact|round]
 *                                      [fail]
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
 * Round 5:
 *   WORLD_SIZE=4  the recursive-doubling plan over 4 members (peers my^1,
 *           my^2); members 1-3 progress, member 0's timer works alone
 *   round   rounded fp32 inputs (the oracle's generator, distinct per member):
 *           every member's result must equal, bit for bit, the oracle's
 *           simulation of the plan (ucg_oracle_reduce_multi, the association
 *           of builtin_recursive.c:158-169) - the default "exact" inputs
 *           (small integers) would hide an association error
 *   fail    just before member 0 goes to sleep, the next device combine call
 *           of its process is armed to fail (ucg_builtin_dev_inject_failure):
 *           the timer thread's combine fails, and member 0's completion
 *           status must be that error (recv_handle_error,
 *           builtin_comp_step.inl:332-333); the other members end with
 *           UCS_ERR_CANCELED as soon as they see member 0 gave up on the op
 *           (round 6), never with a wrong result or a wait timeout
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "ucg_builtin_ops.h"
#include "ucg_builtin_dev.h"
#include "combine_ref.h"          /* the checker (oracle/, test infrastructure) */

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

static int run(char **argv, const char *mode, int round_inputs, int fail);

int main(int argc, char **argv)
{
    return run(argv, argc > 2 ? argv[2] : "host",
               argc > 3 && strcmp(argv[3], "round") == 0,
               argc > 4 && strcmp(argv[4], "fail") == 0);
}

static int run(char **argv, const char *mode, int round_inputs, int fail)
{
    const unsigned rank = (unsigned)atoi(getenv("RANK"));
    const unsigned world = getenv("WORLD_SIZE") ? (unsigned)atoi(getenv("WORLD_SIZE")) : 2;
    const int count = 8192 * 4 / 4;                /* 32 KiB: 133 fragments of 248 B */
    const int staged = strcmp(mode, "staged") == 0, device = strcmp(mode, "device") == 0;
    float *want = malloc(count * sizeof(float));
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
    if (world != 2 && world != 4) {
        fprintf(stderr, "WORLD_SIZE must be 2 or 4\n");
        return 2;
    }
    if (round_inputs) {
        /* every member's input from the oracle's generator; the expected
         * result is the oracle's simulation of the plan over all of them */
        const void *srcs[4];
        float *all = malloc((size_t)world * count * sizeof(float));
        unsigned r;
        for (r = 0; r < world; r++) {
            ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 0xA5A50000u + r, all + (size_t)r * count,
                            count);
            srcs[r] = all + (size_t)r * count;
        }
        memcpy(in, all + (size_t)rank * count, count * sizeof(float));
        ucg_oracle_reduce_multi(ORA_SUM, ORA_F32, want, srcs, world, rank, count);
        free(all);
    } else {
        for (i = 0; i < count; i++) {
            unsigned r;
            in[i] = (float)((int)(rank * 1000 + i) % 4096 - 2048);
            want[i] = 0.0f;
            for (r = 0; r < world; r++) {             /* exact: any order */
                want[i] += (float)((int)(r * 1000 + i) % 4096 - 2048);
            }
        }
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
    if (ucg_builtin_shm_iface_open(argv[1], world, rank, 256, 2, &iface) != UCS_OK ||
        ucg_builtin_lgroup_create(iface, 1, world, rank, cmb, &g) != UCS_OK ||
        ucg_builtin_lcoll_allreduce(g, sbuf, rbuf, count, (void*)1, (void*)1, &c) != UCS_OK) {
        fprintf(stderr, "rank %u: set-up failed\n", rank);
        return 1;
    }
    if ((rank == 0 || device) && ucg_builtin_lgroup_set_async_timer(g, 0.005) != UCS_OK) {
        fprintf(stderr, "timer failed\n");
        return 1;
    }
    ucg_builtin_shm_barrier(iface);
    if (rank != 0) {
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
        if (fail) {
            /* the next device combine call fails - the owner thread makes
             * none from here on, so it is the timer thread's */
            ucg_builtin_dev_inject_failure(1);
        }
        ucg_builtin_shm_barrier(iface);                  /* B2 */
        usleep(1500 * 1000);                             /* the timer thread works alone */
        ucg_builtin_lgroup_async_stats(g, as);
        ucg_builtin_lgroup_stats(g, st4);
        ucg_builtin_combine_stats(cmb, cs);
        printf("{\"mode\": \"%s\", \"world\": %u, \"inputs\": \"%s\", \"fail\": %d, "
               "\"sent_before_sleep\": %llu, \"sent_after_sleep\": %llu, "
               "\"stashed\": %llu, \"timer_resends\": %llu, \"timer_combines\": %llu, "
               "\"host_calls\": %llu, \"device_calls\": %llu, \"staged_steps\": %llu}\n",
               mode, world, round_inputs ? "round" : "exact", fail,
               (unsigned long long)sent_before, (unsigned long long)st4[0],
               (unsigned long long)st4[2], (unsigned long long)as[0],
               (unsigned long long)as[1], (unsigned long long)cs[0],
               (unsigned long long)cs[2], (unsigned long long)cs[4]);
        fflush(stdout);
        if (as[0] == 0 || as[1] == 0 || (!device && !fail && st4[0] < 133)) {
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
        if (memcmp(&out[i], &want[i], sizeof(float)) != 0) {
            fprintf(stderr, "rank %u: element %d: %a != %a (the plan's association)\n", rank, i,
                    out[i], want[i]);
            ok = 0;
            break;
        }
    }
    if (fail) {
        /* member 0 must report the injected error; the others end cleanly or
         * by their wait timeout - a wrong result is caught above */
        /* the error text is the failing thread's (thread-local); the count
         * of injected failures that fired is process-wide */
        printf("{\"rank\": %u, \"status\": %d, \"injected_fired\": %u}\n", rank, (int)st,
               ucg_builtin_dev_inject_failure(0));
        fflush(stdout);
        if (rank == 0 && (st != UCS_ERR_IO_ERROR || ucg_builtin_dev_inject_failure(0) != 1)) {
            fprintf(stderr, "rank 0: status %d, not the injected device error\n", st);
            ok = 0;
        }
        /* member 0 published that it gave up on the op (finish ->
         * shm_abandon): a member still waiting for its fragments ends with
         * UCS_ERR_CANCELED at once, not with its wait timeout - no member
         * has to be timed to meet the others at the last barrier */
        if (rank != 0 && st != UCS_OK && st != UCS_ERR_CANCELED) {
            fprintf(stderr, "rank %u: status %d, not OK or the peer's cancellation\n",
                    rank, st);
            ok = 0;
        }
    } else if (st != UCS_OK) {
        fprintf(stderr, "rank %u: status %d (%s)\n", rank, st,
                (staged || device) ? ucg_builtin_dev_last_error() : "");
        ok = 0;
    }
    if ((st = ucg_builtin_shm_barrier(iface)) != UCS_OK) {
        fprintf(stderr, "rank %u: last barrier: status %d\n", rank, st);
        ok = 0;
    }
    ucg_builtin_lcoll_destroy(c);
    ucg_builtin_lgroup_destroy(g);
    if ((st = ucg_builtin_shm_iface_close(iface)) != UCS_OK) {
        fprintf(stderr, "rank %u: close: status %d\n", rank, st);
        ok = 0;
    }
    ucg_builtin_combine_destroy(cmb);
    if (dctx) {
        ucg_builtin_dev_free(dctx, sbuf);
        ucg_builtin_dev_free(dctx, rbuf);
        ucg_builtin_dev_ctx_destroy(dctx);
    }
    free(in);
    free(out);
    free(want);
    printf("rank %u: %s\n", rank, ok ? "ok" : "FAILED");
    return ok ? 0 : 1;
}

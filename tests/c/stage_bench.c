/*
 * stage_bench.c - row f1's device staging measured from C: one fragmented
 * REDUCE step as the builtin engine drives it (ucg_builtin_dev_stage_begin,
 * one ucg_builtin_dev_combine per arriving AM fragment with the data borrowed
 * for the call, ucg_builtin_dev_stage_end before the next step's send), next
 * to the same step on the host CPU (oracle restatement of reduce_cb_f issued
 * per fragment, 1 thread). fp32 SUM, pageable host buffers as UCX hands them
 * over.
 *
 *   stage_bench [total_bytes] [frag_bytes] [reps]
 *
 * Three device contexts run side by side in one process: the defaults
 * (staged runs <= 64 KiB are read by the kernel from the pinned slot, and
 * stage_end waits on the pinned completion word), one that always copies
 * H2D, and one that waits with hipStreamSynchronize. Every measurement
 * alternates between them rep by rep and reports the median of each, so the
 * A/B is not confounded by box phases (one run per setting is
 * noise).
 *
 * Prints one JSON line; exit 3 if a staged result differs from the oracle.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <time.h>

#include "ucg_builtin_dev.h"
#include "combine_ref.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int staged_step(ucg_builtin_dev_ctx_t *ctx, float *dst, const float *src,
                       size_t total, size_t frag)
{
    size_t off;
    if (ucg_builtin_dev_stage_begin(ctx, dst, total) != UCS_OK) {
        return -1;
    }
    for (off = 0; off < total; off += frag) {
        size_t n = total - off < frag ? total - off : frag;
        if (ucg_builtin_dev_combine(ctx, UCG_DEV_OP_SUM, UCG_DEV_DT_FLOAT32, off,
                                    (const char*)src + off, n / 4) != UCS_OK) {
            return -1;
        }
    }
    return ucg_builtin_dev_stage_end(ctx) == UCS_OK ? 0 : -1;
}

static int cmp_dbl(const void *a, const void *b)
{
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

static double median(double *v, int n)
{
    qsort(v, n, sizeof(*v), cmp_dbl);
    return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

/* one small step into a device recv buffer: stage_begin, one fragment,
 * stage_end (the GPU-aware MPI case); mean us over k steps */
static double small_steps(ucg_builtin_dev_ctx_t *ctx, void *d, const float *src,
                          size_t bytes, int k)
{
    double t0 = 0;
    int i;
    for (i = -20; i < k; i++) {
        if (i == 0) {
            t0 = now_s();
        }
        if (ucg_builtin_dev_stage_begin(ctx, d, bytes) != UCS_OK ||
            ucg_builtin_dev_combine(ctx, UCG_DEV_OP_SUM, UCG_DEV_DT_FLOAT32, 0,
                                    src, bytes / 4) != UCS_OK ||
            ucg_builtin_dev_stage_end(ctx) != UCS_OK) {
            fprintf(stderr, "small step: %s\n", ucg_builtin_dev_last_error());
            return -1;
        }
    }
    return (now_s() - t0) / k * 1e6;
}

#define MAXREPS 64
/* context index: defaults (zero-copy, completion word) / always copy /
 * hipStreamSynchronize completion */
enum { ZC = 0, COPY = 1, SYNC = 2, NCTX = 3 };

int main(int argc, char **argv)
{
    size_t total = argc > 1 ? (size_t)atol(argv[1]) : (64u << 20);
    size_t frag  = argc > 2 ? (size_t)atol(argv[2]) : 8184;
    int reps     = argc > 3 ? atoi(argv[3]) : 5;
    size_t n     = total / 4;
    ucg_builtin_dev_ctx_t *ctx[NCTX];
    float *src, *dst, *want, *ref;
    double t0, t_step[2][MAXREPS], t_cpu[MAXREPS];
    int i, c, ok = 1;

    reps = reps < 1 ? 1 : (reps > MAXREPS ? MAXREPS : reps);
    total = n * 4;
    frag -= frag % 4;
    for (c = 0; c < NCTX; c++) {
        ucg_builtin_dev_ctx_params_t prm = {0, NULL, 0, 0,
                                            c == COPY ? UCG_BUILTIN_DEV_ZCOPY_NEVER : 0,
                                            c == SYNC ? UCG_BUILTIN_DEV_COMPLETION_SYNC :
                                                        UCG_BUILTIN_DEV_COMPLETION_SIGNAL};
        if (ucg_builtin_dev_ctx_create(&prm, &ctx[c]) != UCS_OK) {
            fprintf(stderr, "ctx: %s\n", ucg_builtin_dev_last_error());
            return 1;
        }
    }
    src  = malloc(total);
    dst  = malloc(total);
    want = malloc(total);
    ref  = malloc(total);
    ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 11, src, n);
    ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 12, ref, n);
    memcpy(want, ref, total);
    ucg_oracle_reduce_fragmented(ORA_SUM, ORA_F32, src, want, n, frag);
    for (c = 0; c < 2; c++) {
        memcpy(dst, ref, total);
        if (staged_step(ctx[c], dst, src, total, frag) != 0) {
            fprintf(stderr, "staged step: %s\n", ucg_builtin_dev_last_error());
            return 1;
        }
        ok &= memcmp(dst, want, total) == 0;
    }
    /* the big step, contexts alternated rep by rep, CPU leg in between */
    for (i = 0; i < reps; i++) {
        for (c = 0; c < 2; c++) {
            const int k = (i & 1) ? 1 - c : c;   /* alternate which goes first */
            t0 = now_s();
            staged_step(ctx[k], dst, src, total, frag);
            t_step[k][i] = now_s() - t0;
        }
        t0 = now_s();
        ucg_oracle_reduce_fragmented(ORA_SUM, ORA_F32, src, want, n, frag);
        t_cpu[i] = now_s() - t0;
    }
    /* the same step with the recv buffer registered (hipHostRegister, as a
     * persistent op registers it after MEM_REG_OPT_CNT starts): its H2D and
     * D2H move by DMA. Beside it, the floors of the staged step on this host:
     * copying every borrowed fragment into pinned memory (the ring copy), and
     * the recv buffer's H2D and D2H from registered memory. */
    double t_reg[MAXREPS], t_memcpy[MAXREPS], t_h2d[MAXREPS], t_d2h[MAXREPS];
    {
        char *pin = ucg_builtin_dev_host_alloc(total);
        void *dbuf = ucg_builtin_dev_malloc(ctx[ZC], total);
        size_t off;
        if (pin == NULL || dbuf == NULL ||
            ucg_builtin_dev_host_register(ctx[ZC], dst, total) != UCS_OK) {
            fprintf(stderr, "register: %s\n", ucg_builtin_dev_last_error());
            return 1;
        }
        memcpy(dst, ref, total);
        memcpy(want, ref, total);
        ucg_oracle_reduce_fragmented(ORA_SUM, ORA_F32, src, want, n, frag);
        if (staged_step(ctx[ZC], dst, src, total, frag) != 0) {
            return 1;
        }
        ok &= memcmp(dst, want, total) == 0;
        for (i = 0; i < reps; i++) {
            t0 = now_s();
            staged_step(ctx[ZC], dst, src, total, frag);
            t_reg[i] = now_s() - t0;
            t0 = now_s();
            for (off = 0; off < total; off += frag) {
                size_t m = total - off < frag ? total - off : frag;
                memcpy(pin + off, (const char*)src + off, m);
            }
            t_memcpy[i] = now_s() - t0;
            t0 = now_s();
            ucg_builtin_dev_memcpy(ctx[ZC], dbuf, dst, total);
            t_h2d[i] = now_s() - t0;
            t0 = now_s();
            ucg_builtin_dev_memcpy(ctx[ZC], dst, dbuf, total);
            t_d2h[i] = now_s() - t0;
        }
        ucg_builtin_dev_host_unregister(ctx[ZC], dst);
        ucg_builtin_dev_free(ctx[ZC], dbuf);
        ucg_builtin_dev_host_free(pin);
    }
    /* cost of the memory-kind query the dispatcher makes per step (and per
     * whole-buffer combine): pageable host memory and device memory */
    double mk_host_ns, mk_dev_ns;
    {
        void *d = ucg_builtin_dev_malloc(ctx[ZC], 4096);
        const int k = 100000;
        int acc = 0;
        t0 = now_s();
        for (i = 0; i < k; i++) acc += ucg_builtin_dev_mem_kind(dst + (i & 1023));
        mk_host_ns = (now_s() - t0) / k * 1e9;
        t0 = now_s();
        for (i = 0; i < k; i++) acc += ucg_builtin_dev_mem_kind((char*)d + (i & 1023));
        mk_dev_ns = (now_s() - t0) / k * 1e9;
        ucg_builtin_dev_free(ctx[ZC], d);
        if (acc < 0) return 4;
    }
    uint64_t cnt[2][UCG_BUILTIN_DEV_NCOUNTERS];
    for (c = 0; c < 2; c++) {
        ucg_builtin_dev_counters(ctx[c], cnt[c]);   /* the big steps only */
    }
    /* small steps into a device-resident recv buffer (GPU-aware MPI): 400
     * steps per rep, contexts alternated over `sreps` reps, median per
     * context, plus a parity check of the last small step of each */
    const size_t small[3] = {256, 4096, 65536};
    const int sreps = 7;
    double small_us[NCTX][3], small_lo[NCTX][3], small_hi[NCTX][3];
    {
        int j, r;
        for (j = 0; j < 3; j++) {
            double v[NCTX][7];
            void *d[NCTX];
            for (c = 0; c < NCTX; c++) {
                d[c] = ucg_builtin_dev_malloc(ctx[c], small[j]);
                if (d[c] == NULL) {
                    return 5;
                }
            }
            for (r = 0; r < sreps; r++) {
                for (c = 0; c < NCTX; c++) {
                    const int k = (c + r) % NCTX;   /* rotate which goes first */
                    v[k][r] = small_steps(ctx[k], d[k], src, small[j], 400);
                    if (v[k][r] < 0) {
                        return 5;
                    }
                }
            }
            for (c = 0; c < NCTX; c++) {
                /* d[c] = ref + 421 steps of src (exact: counts of a float
                 * added to itself are compared against the oracle below) */
                float *h = malloc(small[j]), *w = malloc(small[j]);
                size_t e, m = small[j] / 4;
                if (ucg_builtin_dev_memcpy(ctx[c], d[c], ref, small[j]) != UCS_OK ||
                    small_steps(ctx[c], d[c], src, small[j], 1) < 0 ||
                    ucg_builtin_dev_memcpy(ctx[c], h, d[c], small[j]) != UCS_OK) {
                    return 5;
                }
                memcpy(w, ref, small[j]);
                /* small_steps runs 20 warm steps + k: 21 combines for k=1 */
                for (e = 0; e < 21; e++) {
                    ucg_oracle_reduce(ORA_SUM, ORA_F32, src, w, m);
                }
                ok &= memcmp(h, w, small[j]) == 0;
                free(h);
                free(w);
                ucg_builtin_dev_free(ctx[c], d[c]);
                small_lo[c][j] = small_hi[c][j] = v[c][0];
                for (r = 1; r < sreps; r++) {
                    small_lo[c][j] = v[c][r] < small_lo[c][j] ? v[c][r] : small_lo[c][j];
                    small_hi[c][j] = v[c][r] > small_hi[c][j] ? v[c][r] : small_hi[c][j];
                }
                small_us[c][j] = median(v[c], sreps);
            }
        }
    }
    /* where the small-step floor goes, same process: (a) an empty step
     * (stage_begin + stage_end: one stream sync with nothing queued), (b) one
     * device-resident 4 KiB combine + sync (launch + completion wait), each
     * the median of 7 reps of 400 */
    double floor_sync_us, floor_launch_us;
    {
        void *d = ucg_builtin_dev_malloc(ctx[ZC], 8192);
        double v[2][7];
        int r, k;
        if (d == NULL) {
            return 5;
        }
        for (r = 0; r < 7; r++) {
            for (k = -20; k < 400; k++) {
                if (k == 0) t0 = now_s();
                if (ucg_builtin_dev_stage_begin(ctx[ZC], d, 4096) != UCS_OK ||
                    ucg_builtin_dev_stage_end(ctx[ZC]) != UCS_OK) {
                    return 5;
                }
            }
            v[0][r] = (now_s() - t0) / 400 * 1e6;
            for (k = -20; k < 400; k++) {
                if (k == 0) t0 = now_s();
                if (ucg_builtin_dev_reduce(ctx[ZC], UCG_DEV_OP_SUM, UCG_DEV_DT_FLOAT32, d,
                                           (char*)d + 4096, 1024) != UCS_OK ||
                    ucg_builtin_dev_sync(ctx[ZC]) != UCS_OK) {
                    return 5;
                }
            }
            v[1][r] = (now_s() - t0) / 400 * 1e6;
        }
        floor_sync_us   = median(v[0], 7);
        floor_launch_us = median(v[1], 7);
        ucg_builtin_dev_free(ctx[ZC], d);
    }
    {
        double lo[2], hi[2], md[2], cpu_md;
        for (c = 0; c < 2; c++) {
            lo[c] = hi[c] = t_step[c][0];
            for (i = 1; i < reps; i++) {
                lo[c] = t_step[c][i] < lo[c] ? t_step[c][i] : lo[c];
                hi[c] = t_step[c][i] > hi[c] ? t_step[c][i] : hi[c];
            }
            md[c] = median(t_step[c], reps);
        }
        cpu_md = median(t_cpu, reps);
        printf("{\"device_staged_ms_registered_recv\": %.3f, \"fragment_memcpy_ms\": %.3f, "
               "\"h2d_registered_ms\": %.3f, \"d2h_registered_ms\": %.3f, ",
               median(t_reg, reps) * 1e3, median(t_memcpy, reps) * 1e3,
               median(t_h2d, reps) * 1e3, median(t_d2h, reps) * 1e3);
        printf("\"config\": \"f1 staged REDUCE step, fp32 SUM, pageable host buffers\", "
               "\"bytes\": %zu, \"fragment_bytes\": %zu, \"fragments\": %zu, \"reps\": %d, "
               "\"device_staged_ms\": %.3f, \"device_staged_gibs_n\": %.2f, "
               "\"device_staged_ms_range\": [%.3f, %.3f], "
               "\"device_staged_ms_always_copy\": %.3f, "
               "\"device_staged_ms_always_copy_range\": [%.3f, %.3f], "
               "\"cpu_fragmented_ms\": %.3f, \"cpu_fragmented_gibs_n\": %.2f, "
               "\"kernel_launches_total\": %llu, \"h2d_dma_bytes\": %llu, "
               "\"zcopy_read_bytes\": %llu, \"bit_exact\": %s, "
               "\"mem_kind_ns_host\": %.1f, \"mem_kind_ns_device\": %.1f, "
               "\"small_step_us_device_recv\": {\"256\": %.2f, \"4096\": %.2f, "
               "\"65536\": %.2f}, "
               "\"small_step_us_device_recv_always_copy\": {\"256\": %.2f, "
               "\"4096\": %.2f, \"65536\": %.2f}, "
               "\"small_step_us_device_recv_sync_completion\": {\"256\": %.2f, "
               "\"4096\": %.2f, \"65536\": %.2f}, "
               "\"small_step_us_range\": {\"zcopy\": [[%.2f, %.2f], [%.2f, %.2f], "
               "[%.2f, %.2f]], \"copy\": [[%.2f, %.2f], [%.2f, %.2f], [%.2f, %.2f]], "
               "\"sync\": [[%.2f, %.2f], [%.2f, %.2f], [%.2f, %.2f]]}, "
               "\"small_step_timing\": \"median of %d alternating reps of 400 steps "
               "per context, one process\", \"floor_empty_step_us\": %.2f, "
               "\"floor_device_reduce_4k_plus_sync_us\": %.2f}\n",
               total, frag, (total + frag - 1) / frag, reps,
               md[ZC] * 1e3, total / md[ZC] / 1073741824.0, lo[ZC] * 1e3, hi[ZC] * 1e3,
               md[COPY] * 1e3, lo[COPY] * 1e3, hi[COPY] * 1e3,
               cpu_md * 1e3, total / cpu_md / 1073741824.0,
               (unsigned long long)cnt[ZC][0], (unsigned long long)cnt[ZC][2],
               (unsigned long long)cnt[ZC][4], ok ? "true" : "false",
               mk_host_ns, mk_dev_ns,
               small_us[ZC][0], small_us[ZC][1], small_us[ZC][2],
               small_us[COPY][0], small_us[COPY][1], small_us[COPY][2],
               small_us[SYNC][0], small_us[SYNC][1], small_us[SYNC][2],
               small_lo[ZC][0], small_hi[ZC][0], small_lo[ZC][1], small_hi[ZC][1],
               small_lo[ZC][2], small_hi[ZC][2],
               small_lo[COPY][0], small_hi[COPY][0], small_lo[COPY][1], small_hi[COPY][1],
               small_lo[COPY][2], small_hi[COPY][2],
               small_lo[SYNC][0], small_hi[SYNC][0], small_lo[SYNC][1], small_hi[SYNC][1],
               small_lo[SYNC][2], small_hi[SYNC][2], sreps, floor_sync_us,
               floor_launch_us);
    }
    for (c = 0; c < NCTX; c++) {
        ucg_builtin_dev_ctx_destroy(ctx[c]);
    }
    free(src);
    free(dst);
    free(want);
    free(ref);
    return ok ? 0 : 3;
}

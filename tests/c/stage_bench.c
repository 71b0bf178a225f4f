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
 * Prints one JSON line; exit 3 if the staged result differs from the oracle.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
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

int main(int argc, char **argv)
{
    size_t total = argc > 1 ? (size_t)atol(argv[1]) : (64u << 20);
    size_t frag  = argc > 2 ? (size_t)atol(argv[2]) : 8184;
    int reps     = argc > 3 ? atoi(argv[3]) : 5;
    size_t n     = total / 4;
    ucg_builtin_dev_ctx_params_t prm = {0, NULL, 0, 0};
    ucg_builtin_dev_ctx_t *ctx;
    float *src, *dst, *want;
    double t0, t_dev = 1e30, t_cpu = 1e30;
    int i, ok;

    total = n * 4;
    frag -= frag % 4;
    if (ucg_builtin_dev_ctx_create(&prm, &ctx) != UCS_OK) {
        fprintf(stderr, "ctx: %s\n", ucg_builtin_dev_last_error());
        return 1;
    }
    src  = malloc(total);
    dst  = malloc(total);
    want = malloc(total);
    ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 11, src, n);
    ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 12, want, n);
    memcpy(dst, want, total);
    ucg_oracle_reduce_fragmented(ORA_SUM, ORA_F32, src, want, n, frag);
    if (staged_step(ctx, dst, src, total, frag) != 0) {
        fprintf(stderr, "staged step: %s\n", ucg_builtin_dev_last_error());
        return 1;
    }
    ok = memcmp(dst, want, total) == 0;
    for (i = 0; i < reps; i++) {
        t0 = now_s();
        staged_step(ctx, dst, src, total, frag);
        t0 = now_s() - t0;
        t_dev = t0 < t_dev ? t0 : t_dev;
        t0 = now_s();
        ucg_oracle_reduce_fragmented(ORA_SUM, ORA_F32, src, want, n, frag);
        t0 = now_s() - t0;
        t_cpu = t0 < t_cpu ? t0 : t_cpu;
    }
    /* cost of the memory-kind query the dispatcher makes per step (and per
     * whole-buffer combine): pageable host memory and device memory */
    double mk_host_ns, mk_dev_ns;
    {
        void *d = ucg_builtin_dev_malloc(ctx, 4096);
        const int k = 100000;
        int acc = 0;
        t0 = now_s();
        for (i = 0; i < k; i++) acc += ucg_builtin_dev_mem_kind(dst + (i & 1023));
        mk_host_ns = (now_s() - t0) / k * 1e9;
        t0 = now_s();
        for (i = 0; i < k; i++) acc += ucg_builtin_dev_mem_kind((char*)d + (i & 1023));
        mk_dev_ns = (now_s() - t0) / k * 1e9;
        ucg_builtin_dev_free(ctx, d);
        if (acc < 0) return 4;
    }
    /* small steps into a device-resident recv buffer (GPU-aware MPI): one
     * fragment per step, stage_begin .. stage_end, mean over 2000 steps */
    const size_t small[3] = {256, 4096, 65536};
    double small_us[3];
    uint64_t c[4];
    ucg_builtin_dev_counters(ctx, c);   /* launches of the 64 MiB steps */
    {
        int j;
        for (j = 0; j < 3; j++) {
            const int k = 2000;
            void *d = ucg_builtin_dev_malloc(ctx, small[j]);
            if (d == NULL || ucg_builtin_dev_memcpy(ctx, d, dst, small[j]) != UCS_OK) {
                return 5;
            }
            for (i = -50; i < k; i++) {
                if (i == 0) {
                    t0 = now_s();
                }
                if (ucg_builtin_dev_stage_begin(ctx, d, small[j]) != UCS_OK ||
                    ucg_builtin_dev_combine(ctx, UCG_DEV_OP_SUM, UCG_DEV_DT_FLOAT32, 0,
                                            src, small[j] / 4) != UCS_OK ||
                    ucg_builtin_dev_stage_end(ctx) != UCS_OK) {
                    fprintf(stderr, "small step: %s\n", ucg_builtin_dev_last_error());
                    return 5;
                }
            }
            small_us[j] = (now_s() - t0) / k * 1e6;
            ucg_builtin_dev_free(ctx, d);
        }
    }
    {
        const char *z = getenv("UCX_BUILTIN_DEV_ZCOPY_BYTES");
        printf("{\"config\": \"f1 staged REDUCE step, fp32 SUM, pageable host buffers\", "
               "\"bytes\": %zu, \"fragment_bytes\": %zu, \"fragments\": %zu, "
               "\"device_staged_ms\": %.3f, \"device_staged_gibs_n\": %.2f, "
               "\"cpu_fragmented_ms\": %.3f, \"cpu_fragmented_gibs_n\": %.2f, "
               "\"kernel_launches_total\": %llu, \"bit_exact\": %s, "
               "\"mem_kind_ns_host\": %.1f, \"mem_kind_ns_device\": %.1f, "
               "\"small_step_us_device_recv\": {\"256\": %.2f, \"4096\": %.2f, "
               "\"65536\": %.2f}, \"zcopy_bytes\": \"%s\"}\n",
               total, frag, (total + frag - 1) / frag, t_dev * 1e3,
               total / t_dev / 1073741824.0, t_cpu * 1e3, total / t_cpu / 1073741824.0,
               (unsigned long long)c[0], ok ? "true" : "false", mk_host_ns, mk_dev_ns,
               small_us[0], small_us[1], small_us[2], z ? z : "default");
    }
    ucg_builtin_dev_ctx_destroy(ctx);
    free(src);
    free(dst);
    free(want);
    return ok ? 0 : 3;
}

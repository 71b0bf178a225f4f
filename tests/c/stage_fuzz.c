/*
 * stage_fuzz.c - row f1's fragment aggregator fuzzed from C against the
 * oracle: random dtype x op, step length, fragment size, number of
 * interleaved senders (a fan-in step with ep_cnt > 1), arrival order, recv
 * buffer kind (pageable or pinned host memory at any element offset, or
 * device memory; the last two end their step on the completion word) and
 * staging ring geometry (small slots and shallow rings force the flush,
 * clash and slot-reuse paths of ucg_builtin_dev_combine).
 *
 * Every fragment is handed over the way the AM handler does
 * (builtin/ops/builtin_comp_step.inl:443-449): the payload lives in a
 * buffer that is poisoned and freed as soon as the combine returns, so a
 * shim that kept the borrowed pointer reads garbage (or, in the sanitizer
 * build, a freed block). The expected result applies the oracle's
 * reduce_cb_f restatement per fragment in arrival order, so the check is
 * bit-exact for every dtype and op, NaN payloads included.
 *
 *   stage_fuzz [cases] [seed]
 *
 * A quarter of the cases take the whole-buffer form instead
 * (ucg_builtin_dev_combine_host): src and dst each pageable, pinned or
 * device memory at any element offset.
 *
 * Prints one JSON line; exit 3 on the first mismatch (with its case).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ucg_builtin_dev.h"
#include "combine_ref.h"

static uint64_t g_rng;

static uint64_t rnd(void)
{
    g_rng += 0x9E3779B97F4A7C15ull;
    return ucg_oracle_splitmix64(g_rng);
}

static size_t rnd_in(size_t lo, size_t hi)      /* inclusive */
{
    return lo + (size_t)(rnd() % (hi - lo + 1));
}

typedef struct {
    unsigned sender;
    size_t   off;       /* bytes into the step buffer */
    size_t   bytes;
} frag_t;

static int run_case(ucg_builtin_dev_ctx_t *ctx, int c, int *kinds)
{
    int dt, op;
    do {
        dt = (int)rnd_in(0, UCG_DEV_DT_LAST - 1);
        op = (int)rnd_in(0, UCG_DEV_OP_LAST - 1);
    } while (!ucg_oracle_is_supported(dt, op));
    const size_t sz      = ucg_oracle_dtype_size(dt);
    const size_t count   = rnd() % 4 == 0 ? rnd_in(1, 64) : rnd_in(1, 300000 / sz);
    const size_t bytes   = count * sz;
    const unsigned nsend = (unsigned)rnd_in(1, 4);
    const size_t frag    = sz * rnd_in(1, rnd() % 2 ? 64 : 16384 / sz);
    const int recv_kind  = (int)(rnd() % 3);   /* 0 pageable, 1 device, 2 pinned */
    const int dev_recv   = recv_kind == 1;
    const size_t pad     = sz * rnd_in(0, 16 / sz + 1);  /* recv offset in elements */
    const int dist       = (int)rnd_in(0, ORA_DIST_LAST - 1);
    const int shuffle    = rnd() % 4 == 0;  /* reorder within a sender too */
    char **srcs = calloc(nsend, sizeof(*srcs));
    char *host_acc = recv_kind == 2 ? ucg_builtin_dev_host_alloc(pad + bytes + 1)
                                    : malloc(pad + bytes + 1);
    char *want = malloc(bytes + 1);
    char *got = malloc(bytes + 1);
    void *dbuf = NULL;
    size_t nfr_per = (bytes + frag - 1) / frag, nfr = nsend * nfr_per, i, k;
    frag_t *fr = calloc(nfr, sizeof(*fr));
    size_t *next = calloc(nsend, sizeof(*next));
    int ok = 1;

    if (host_acc == NULL) {
        fprintf(stderr, "case %d: recv buffer: %s\n", c, ucg_builtin_dev_last_error());
        return -1;
    }
    kinds[recv_kind]++;
    for (k = 0; k < nsend; k++) {
        srcs[k] = malloc(bytes + 1);
        ucg_oracle_fill(dt, dist, 0xF0220000ull + 97ull * c + k, srcs[k], count);
    }
    ucg_oracle_fill(dt, dist, 0xF0230000ull + c, want, count);
    memcpy(host_acc + pad, want, bytes);
    if (dev_recv) {
        dbuf = ucg_builtin_dev_malloc(ctx, pad + bytes);
        if (dbuf == NULL ||
            ucg_builtin_dev_memcpy(ctx, (char*)dbuf + pad, want, bytes) != UCS_OK ||
            ucg_builtin_dev_sync(ctx) != UCS_OK) {
            fprintf(stderr, "case %d: device recv buffer: %s\n", c,
                    ucg_builtin_dev_last_error());
            return -1;
        }
    }

    /* arrival order: senders interleaved at random, each sender's fragments
     * in offset order (one ordered AM stream per peer) unless shuffled */
    for (k = 0; k < nsend; k++) {
        for (i = 0; i < nfr_per; i++) {
            frag_t *f = &fr[k * nfr_per + i];
            f->sender = (unsigned)k;
            f->off    = i * frag;
            f->bytes  = bytes - f->off < frag ? bytes - f->off : frag;
        }
    }
    if (shuffle) {
        for (i = nfr; i > 1; i--) {
            size_t j = rnd() % i;
            frag_t t = fr[i - 1];
            fr[i - 1] = fr[j];
            fr[j] = t;
        }
    } else {
        /* merge the per-sender lists in a random interleaving */
        frag_t *m = calloc(nfr, sizeof(*m));
        for (i = 0; i < nfr; i++) {
            unsigned s;
            do {
                s = (unsigned)rnd_in(0, nsend - 1);
            } while (next[s] == nfr_per);
            m[i] = fr[s * nfr_per + next[s]++];
        }
        free(fr);
        fr = m;
    }

    if (ucg_builtin_dev_stage_begin(ctx, dev_recv ? (char*)dbuf + pad : host_acc + pad,
                                    bytes) != UCS_OK) {
        fprintf(stderr, "case %d: stage_begin: %s\n", c, ucg_builtin_dev_last_error());
        return -1;
    }
    for (i = 0; i < nfr; i++) {
        const frag_t *f = &fr[i];
        /* the borrowed AM payload: valid for the duration of the call only */
        char *am = malloc(f->bytes);
        memcpy(am, srcs[f->sender] + f->off, f->bytes);
        if (ucg_builtin_dev_combine(ctx, (ucg_dev_op_t)op, (ucg_dev_dtype_t)dt, f->off,
                                    am, f->bytes / sz) != UCS_OK) {
            fprintf(stderr, "case %d: combine: %s\n", c, ucg_builtin_dev_last_error());
            return -1;
        }
        memset(am, 0xA5, f->bytes);
        free(am);
        ucg_oracle_reduce(op, dt, srcs[f->sender] + f->off, want + f->off, f->bytes / sz);
    }
    if (ucg_builtin_dev_stage_end(ctx) != UCS_OK) {
        fprintf(stderr, "case %d: stage_end: %s\n", c, ucg_builtin_dev_last_error());
        return -1;
    }
    if (dev_recv) {
        if (ucg_builtin_dev_memcpy(ctx, got, (char*)dbuf + pad, bytes) != UCS_OK ||
            ucg_builtin_dev_sync(ctx) != UCS_OK) {
            return -1;
        }
        ucg_builtin_dev_free(ctx, dbuf);
    } else {
        memcpy(got, host_acc + pad, bytes);
    }
    if (memcmp(got, want, bytes) != 0) {
        for (i = 0; i < bytes && got[i] == want[i]; i++) {
        }
        fprintf(stderr, "case %d MISMATCH: dt=%d op=%d count=%zu frag=%zu senders=%u "
                "recv_kind=%d pad=%zu shuffle=%d first bad byte %zu\n", c, dt, op,
                count, frag, nsend, recv_kind, pad, shuffle, i);
        ok = 0;
    }
    for (k = 0; k < nsend; k++) {
        free(srcs[k]);
    }
    free(srcs);
    if (recv_kind == 2) {
        ucg_builtin_dev_host_free(host_acc);
    } else {
        free(host_acc);
    }
    free(want);
    free(got);
    free(fr);
    free(next);
    return ok;
}

/* Whole-buffer form (ucg_builtin_dev_combine_host, the reduce_cb_f call
 * shape): src and dst each pageable, pinned or device memory, at any
 * element offset; lengths cross the ring's chunk boundaries. */
static int run_whole(ucg_builtin_dev_ctx_t *ctx, int c, int *kinds)
{
    int dt, op;
    do {
        dt = (int)rnd_in(0, UCG_DEV_DT_LAST - 1);
        op = (int)rnd_in(0, UCG_DEV_OP_LAST - 1);
    } while (!ucg_oracle_is_supported(dt, op));
    const size_t sz    = ucg_oracle_dtype_size(dt);
    const size_t count = rnd() % 4 == 0 ? rnd_in(1, 64) : rnd_in(1, 400000 / sz);
    const size_t bytes = count * sz;
    const int dist     = (int)rnd_in(0, ORA_DIST_LAST - 1);
    const int kind[2]  = {(int)rnd_in(0, 2), (int)rnd_in(0, 2)};  /* src, dst */
    const size_t pad[2] = {sz * rnd_in(0, 16 / sz + 1), sz * rnd_in(0, 16 / sz + 1)};
    char *host[2], *base[2], *want = malloc(bytes + 1), *got = malloc(bytes + 1);
    int j, ok = 1;

    ucg_oracle_fill(dt, dist, 0xF0240000ull + c, want, count);   /* dst */
    for (j = 0; j < 2; j++) {
        host[j] = malloc(bytes + 1);
        ucg_oracle_fill(dt, dist, j ? 0xF0240000ull + c : 0xF0250000ull + c, host[j],
                        count);
        kinds[kind[j]]++;
        base[j] = kind[j] == 0 ? malloc(pad[j] + bytes)
                : kind[j] == 1 ? ucg_builtin_dev_host_alloc(pad[j] + bytes)
                               : ucg_builtin_dev_malloc(ctx, pad[j] + bytes);
        if (base[j] == NULL) {
            fprintf(stderr, "case %d: allocation: %s\n", c, ucg_builtin_dev_last_error());
            return -1;
        }
        if (kind[j] == 2) {
            if (ucg_builtin_dev_memcpy(ctx, base[j] + pad[j], host[j], bytes) != UCS_OK) {
                return -1;
            }
        } else {
            memcpy(base[j] + pad[j], host[j], bytes);
        }
    }
    ucg_oracle_reduce(op, dt, host[0], want, count);
    if (ucg_builtin_dev_combine_host(ctx, (ucg_dev_op_t)op, (ucg_dev_dtype_t)dt,
                                     base[1] + pad[1], base[0] + pad[0], count) != UCS_OK) {
        fprintf(stderr, "case %d: combine_host: %s\n", c, ucg_builtin_dev_last_error());
        return -1;
    }
    if (kind[1] == 2) {
        if (ucg_builtin_dev_memcpy(ctx, got, base[1] + pad[1], bytes) != UCS_OK) {
            return -1;
        }
    } else {
        memcpy(got, base[1] + pad[1], bytes);
    }
    if (memcmp(got, want, bytes) != 0) {
        fprintf(stderr, "case %d MISMATCH (whole buffer): dt=%d op=%d count=%zu "
                "src kind %d pad %zu, dst kind %d pad %zu\n", c, dt, op, count,
                kind[0], pad[0], kind[1], pad[1]);
        ok = 0;
    }
    for (j = 0; j < 2; j++) {
        if (kind[j] == 0) {
            free(base[j]);
        } else if (kind[j] == 1) {
            ucg_builtin_dev_host_free(base[j]);
        } else {
            ucg_builtin_dev_free(ctx, base[j]);
        }
        free(host[j]);
    }
    free(want);
    free(got);
    return ok;
}

int main(int argc, char **argv)
{
    const int cases = argc > 1 ? atoi(argv[1]) : 200;
    g_rng = argc > 2 ? strtoull(argv[2], NULL, 0) : 0x5EEDF022ull;
    /* ring geometries: tiny slots (a fragment spans slots, runs fill
     * quickly), a shallow ring (slot reuse waits on the stream), default;
     * each with the default zero-copy threshold (runs <= 64 KiB are read by
     * the kernel from the pinned slot: every run of the 4 KiB and 64 KiB
     * geometries) and again with zero-copy off (every run copied H2D), so
     * both flush paths see the clash and slot-reuse orderings */
    const size_t slot_bytes[] = {4096, 65536, 0, 4096, 65536, 0};
    const unsigned slots[]    = {2, 3, 0, 2, 3, 0};
    const size_t zcopy[]      = {0, 0, 0, UCG_BUILTIN_DEV_ZCOPY_NEVER,
                                 UCG_BUILTIN_DEV_ZCOPY_NEVER, UCG_BUILTIN_DEV_ZCOPY_NEVER};
    const int ngeo = 6;
    int kinds[3] = {0, 0, 0}, whole_kinds[3] = {0, 0, 0}, done = 0, whole = 0, g, c;
    int by_path[2] = {0, 0};
    uint64_t zc_bytes = 0, dma_bytes = 0, signal_waits = 0;

    for (g = 0; g < ngeo; g++) {
        /* odd geometries wait with hipStreamSynchronize, even ones on the
         * completion word: both stage_end paths are fuzzed */
        ucg_builtin_dev_ctx_params_t prm = {0, NULL, slot_bytes[g], slots[g], zcopy[g],
                                            (g & 1) ? UCG_BUILTIN_DEV_COMPLETION_SYNC :
                                                      UCG_BUILTIN_DEV_COMPLETION_SIGNAL};
        ucg_builtin_dev_ctx_t *ctx;
        if (ucg_builtin_dev_ctx_create(&prm, &ctx) != UCS_OK) {
            fprintf(stderr, "ctx: %s\n", ucg_builtin_dev_last_error());
            return 1;
        }
        for (c = g; c < cases; c += ngeo) {
            const int w = rnd() % 4 == 0;
            int r = w ? run_whole(ctx, c, whole_kinds) : run_case(ctx, c, kinds);
            whole += w;
            if (r < 0) {
                return 1;
            }
            if (r == 0) {
                return 3;
            }
            done++;
            by_path[zcopy[g] == UCG_BUILTIN_DEV_ZCOPY_NEVER]++;
            if (done % 250 == 0) {   /* progress for long runs */
                fprintf(stderr, "stage_fuzz: %d cases bit-exact\n", done);
            }
        }
        {
            uint64_t cnt[UCG_BUILTIN_DEV_NCOUNTERS];
            ucg_builtin_dev_counters(ctx, cnt);
            dma_bytes += cnt[2];
            zc_bytes  += cnt[4];
            signal_waits += cnt[5];
            if ((g & 1) && cnt[5] != 0) {
                fprintf(stderr, "geometry %d: sync completion but %llu signal waits\n", g,
                        (unsigned long long)cnt[5]);
                return 3;
            }
            if (zcopy[g] == UCG_BUILTIN_DEV_ZCOPY_NEVER && cnt[4] != 0) {
                fprintf(stderr, "geometry %d: zero-copy off but %llu bytes read in "
                        "place\n", g, (unsigned long long)cnt[4]);
                return 3;
            }
        }
        ucg_builtin_dev_ctx_destroy(ctx);
    }
    printf("{\"harness\": \"stage_fuzz\", \"cases\": %d, \"host_recv\": %d, "
           "\"device_recv\": %d, \"pinned_recv\": %d, \"whole_buffer\": %d, \"whole_operands\": "
           "{\"pageable\": %d, \"pinned\": %d, \"device\": %d}, "
           "\"cases_zcopy_default\": %d, \"cases_zcopy_off\": %d, "
           "\"h2d_dma_bytes\": %llu, \"zcopy_read_bytes\": %llu, "
           "\"stage_end_signal_waits\": %llu, \"bit_exact\": true}\n",
           done, kinds[0], kinds[1], kinds[2], whole, whole_kinds[0], whole_kinds[1], whole_kinds[2],
           by_path[0], by_path[1], (unsigned long long)dma_bytes,
           (unsigned long long)zc_bytes, (unsigned long long)signal_waits);
    return 0;
}

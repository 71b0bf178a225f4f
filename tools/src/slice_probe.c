/*
 * slice_probe.c - what makes kernels of several processes on one GPU take
 * ~37 us quantized durations? Round 4 saw it in the C1
 * device-buffer allreduce with the engine's pools in shareable (HIP VMM)
 * memory: k_reduce_multi and k_signal (which reads no imported memory) took
 * whole multiples of ~37 us, against 2.2 / 0.6 us with hipMalloc pools.
 *
 * NP processes on the one GPU, each with a device context of the product
 * library (the engine's setup: one created stream, the pinned completion
 * word), one 2 MiB buffer of its own, and the engine's per-op pattern on it:
 * a 4 KiB 4-operand fold (ucg_builtin_dev_reduce_multi) then
 * ucg_builtin_dev_complete (k_signal + spin on the word). Modes:
 *   mem  plain | shareable   the own buffer (ucg_builtin_dev_malloc[_shareable])
 *        mixed               rank 0 plain, the others shareable
 *        freed               a shareable allocation made and freed first, then
 *                            plain buffers (does the effect outlive it?)
 *   imp  none | held | read  peers' buffers not imported / imported but the
 *                            fold reads this process's own memory / the fold
 *                            reads the imports (the engine's pattern)
 *   act  all | one           every process runs the loop / only rank 0 does,
 *                            the others sleep holding their setup
 * Each process prints one JSON line: latency per op (p10 .. max), the KFD's
 * per-process queue-eviction time (/sys/class/kfd/kfd/proc/<pid>/stats_*
 * /evicted_ms) across the loop, and its queues as the KFD lists them
 * (/sys/class/kfd/kfd/proc/<pid>/queues/<id>/type).
 *
 *   slice_probe <dir> <rank> <np> <mem> <imp> <act> <iters>
 *
 * Processes meet through files in <dir> (keys and barriers). Started by
 * scripts/slice_probe.py. Built by `make -C tools/src` into tools/ (not part
 * of the product).
 */
#define _GNU_SOURCE
#include <dirent.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "ucg_builtin_dev.h"

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static void die(const char *what, int st)
{
    printf("{\"error\": \"%s (%d): %s\"}\n", what, st, ucg_builtin_dev_last_error());
    fflush(stdout);
    exit(1);
}

static void put_file(const char *dir, const char *name, const void *p, size_t n)
{
    char tmp[512], fin[512];
    snprintf(tmp, sizeof(tmp), "%s/.%s.tmp", dir, name);
    snprintf(fin, sizeof(fin), "%s/%s", dir, name);
    FILE *f = fopen(tmp, "wb");
    if (f == NULL || fwrite(p, 1, n, f) != n || fclose(f) != 0 || rename(tmp, fin) != 0) {
        die("put_file", -1);
    }
}

static int get_file(const char *dir, const char *name, void *p, size_t n)
{
    char fin[512];
    snprintf(fin, sizeof(fin), "%s/%s", dir, name);
    FILE *f = fopen(fin, "rb");
    if (f == NULL) {
        return 0;
    }
    const size_t r = fread(p, 1, n, f);
    fclose(f);
    return r == n;
}

/* every process has put `<tag>_<rank>` (60 s at most) */
static void barrier(const char *dir, const char *tag, int rank, int np)
{
    char name[128];
    char one = 1;
    snprintf(name, sizeof(name), "%s_%d", tag, rank);
    put_file(dir, name, &one, 1);
    const double t0 = now_us();
    for (int r = 0; r < np; r++) {
        snprintf(name, sizeof(name), "%s_%d", tag, r);
        while (!get_file(dir, name, &one, 1)) {
            if (now_us() - t0 > 60e6) {
                die("barrier timeout", r);
            }
            usleep(200);
        }
    }
}

/* sum of stats_<gpuid>/evicted_ms over the process's GPUs (-1: unreadable) */
static long evicted_ms(void)
{
    char path[256];
    snprintf(path, sizeof(path), "/sys/class/kfd/kfd/proc/%d", (int)getpid());
    DIR *d = opendir(path);
    if (d == NULL) {
        return -1;
    }
    long sum = -1;
    struct dirent *e;
    while ((e = readdir(d)) != NULL) {
        if (strncmp(e->d_name, "stats_", 6) != 0) {
            continue;
        }
        char f[600];
        snprintf(f, sizeof(f), "%s/%s/evicted_ms", path, e->d_name);
        FILE *fp = fopen(f, "r");
        long v;
        if (fp && fscanf(fp, "%ld", &v) == 1) {
            sum = (sum < 0 ? 0 : sum) + v;
        }
        if (fp) {
            fclose(fp);
        }
    }
    closedir(d);
    return sum;
}

/* the process's queues as the KFD lists them: "n:type,type,..." */
static void queues(char *out, size_t max)
{
    char path[256];
    snprintf(path, sizeof(path), "/sys/class/kfd/kfd/proc/%d/queues", (int)getpid());
    DIR *d = opendir(path);
    if (d == NULL) {
        snprintf(out, max, "unreadable");
        return;
    }
    int n = 0;
    size_t len = 0;
    out[0] = 0;
    struct dirent *e;
    while ((e = readdir(d)) != NULL) {
        if (e->d_name[0] == '.') {
            continue;
        }
        char f[600], t[32] = "?";
        snprintf(f, sizeof(f), "%s/%s/type", path, e->d_name);
        FILE *fp = fopen(f, "r");
        if (fp) {
            if (fscanf(fp, "%31s", t) != 1) {
                strcpy(t, "?");
            }
            fclose(fp);
        }
        n++;
        len += (size_t)snprintf(out + len, len < max ? max - len : 0, "%s%s", n > 1 ? "," : "", t);
    }
    closedir(d);
    char tmp[600];
    snprintf(tmp, sizeof(tmp), "%d:%.500s", n, out);
    snprintf(out, max, "%.*s", (int)(max - 1), tmp);
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

int main(int argc, char **argv)
{
    if (argc < 8) {
        fprintf(stderr, "usage: slice_probe <dir> <rank> <np> <mem> <imp> <act> <iters>\n");
        return 2;
    }
    const char *dir = argv[1];
    const int rank = atoi(argv[2]), np = atoi(argv[3]);
    const char *mem = argv[4];
    const int shareable = strcmp(mem, "shareable") == 0 || (strcmp(mem, "mixed") == 0 && rank > 0);
    const char *imp = argv[5];
    const int act_all = strcmp(argv[6], "all") == 0;
    const int iters = atoi(argv[7]);
    const int nops = 4;                       /* the fold's operands */
    const size_t count = 1024;                /* 4 KiB fp32 */
    if (np < 1 || np > 16 || rank < 0 || rank >= np || iters < 1) {
        return 2;
    }

    ucg_builtin_dev_ctx_params_t prm;
    memset(&prm, 0, sizeof(prm));
    prm.device = 0;
    ucg_builtin_dev_ctx_t *ctx;
    int st = ucg_builtin_dev_ctx_create(&prm, &ctx);
    if (st != UCS_OK) {
        die("ctx_create", st);
    }
    char qs_start[512];
    queues(qs_start, sizeof(qs_start));
    const size_t bytes = (size_t)2 << 20;
    if (strcmp(mem, "freed") == 0) {
        void *t = ucg_builtin_dev_malloc_shareable(ctx, bytes);
        if (t == NULL) {
            die("malloc_shareable", -4);
        }
        ucg_builtin_dev_free(ctx, t);
    }
    char *own = shareable ? ucg_builtin_dev_malloc_shareable(ctx, bytes)
                          : ucg_builtin_dev_malloc(ctx, bytes);
    char *out = ucg_builtin_dev_malloc(ctx, bytes);
    if (own == NULL || out == NULL) {
        die("malloc", -4);
    }
    st = ucg_builtin_dev_fill(ctx, UCG_DEV_DT_FLOAT32, UCG_DEV_DIST_EXACT, 0x5EED + rank, own,
                              bytes / 4);
    if (st != UCS_OK || (st = ucg_builtin_dev_sync(ctx)) != UCS_OK) {
        die("fill", st);
    }

    /* keys: every process exports its buffer; imports per mode */
    char blob[UCG_BUILTIN_DEV_IPC_HANDLE_BYTES], name[64];
    void *peer[16] = {0};
    if (strcmp(imp, "none") != 0) {
        st = ucg_builtin_dev_ipc_export(ctx, own, blob);
        if (st != UCS_OK) {
            die("ipc_export", st);
        }
        snprintf(name, sizeof(name), "key_%d", rank);
        put_file(dir, name, blob, sizeof(blob));
    }
    barrier(dir, "keys", rank, np);
    if (strcmp(imp, "none") != 0) {
        for (int p = 0; p < np; p++) {
            if (p == rank) {
                continue;
            }
            snprintf(name, sizeof(name), "key_%d", p);
            if (!get_file(dir, name, blob, sizeof(blob))) {
                die("key file", p);
            }
            st = ucg_builtin_dev_ipc_import(ctx, blob, &peer[p]);
            if (st != UCS_OK) {
                die("ipc_import", st);
            }
        }
    }
    /* the fold's operands: own buffer at 4 offsets, or own + up to 3 imports */
    const void *srcs[4];
    for (int m = 0; m < nops; m++) {
        srcs[m] = own + (size_t)m * 4096;
    }
    if (strcmp(imp, "read") == 0) {
        int m = 1;
        for (int p = 0; p < np && m < nops; p++) {
            if (p != rank) {
                srcs[m++] = peer[p];
            }
        }
    }
    char qs_setup[512];
    queues(qs_setup, sizeof(qs_setup));
    barrier(dir, "setup", rank, np);

    const int active = act_all || rank == 0;
    double *lat = calloc((size_t)iters, sizeof(double));
    long ev0 = evicted_ms();
    const double t_start = now_us();
    if (active) {
        for (int i = -50; i < iters; i++) {          /* 50 warm-up ops */
            const double t0 = now_us();
            st = ucg_builtin_dev_reduce_multi(ctx, UCG_DEV_OP_SUM, UCG_DEV_DT_FLOAT32, out, srcs,
                                              nops, 0, count);
            if (st == UCS_OK) {
                st = ucg_builtin_dev_complete(ctx);
            }
            if (st != UCS_OK) {
                die("fold", st);
            }
            if (i >= 0) {
                lat[i] = now_us() - t0;
            }
        }
    }
    const double wall = now_us() - t_start;
    long ev1 = evicted_ms();
    char qs_run[512];
    queues(qs_run, sizeof(qs_run));
    barrier(dir, "done", rank, np);          /* nobody unmaps while a peer reads */

    if (active) {
        qsort(lat, (size_t)iters, sizeof(double), cmp_d);
    }
#define Q(f) (active ? lat[(size_t)((iters - 1) * (f))] : 0.0)
    printf("{\"rank\": %d, \"np\": %d, \"mem\": \"%s\", \"imp\": \"%s\", \"act\": \"%s\", "
           "\"active\": %d, \"iters\": %d, \"op_us\": {\"p10\": %.2f, \"p50\": %.2f, "
           "\"p90\": %.2f, \"p99\": %.2f, \"max\": %.2f}, \"wall_ms\": %.1f, "
           "\"evicted_ms_before\": %ld, \"evicted_ms_after\": %ld, "
           "\"queues_after_ctx\": \"%s\", \"queues_after_setup\": \"%s\", "
           "\"queues_after_loop\": \"%s\"}\n",
           rank, np, argv[4], imp, argv[6], active, iters, Q(0.10), Q(0.50), Q(0.90), Q(0.99),
           Q(1.0), wall * 1e-3, ev0, ev1, qs_start, qs_setup, qs_run);
#undef Q
    fflush(stdout);
    for (int p = 0; p < np; p++) {
        if (peer[p]) {
            ucg_builtin_dev_ipc_release(ctx, peer[p]);
        }
    }
    barrier(dir, "released", rank, np);      /* no import outlives its exporter */
    ucg_builtin_dev_free(ctx, own);
    ucg_builtin_dev_free(ctx, out);
    ucg_builtin_dev_ctx_destroy(ctx);
    free(lat);
    return 0;
}

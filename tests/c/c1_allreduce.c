/*
 * c1_allreduce.c - BASELINE config 1: an N-process loopback allreduce of
 * 4 KiB fp32 SUM through the builtin operation engine (libucg_builtin.so)
 * over the shared-memory transport, combine on the host callback.
 *
 *   RANK=r WORLD_SIZE=n c1_allreduce <shm-name> [iters] [max_short] [count]
 *
 * C1_DEVICE_STAGING=1 forces every combine onto the GPU (staged steps).
 * C1_DEVICE_BUFFERS=1 gives the engine device buffers (GPU rank % count): the
 * plan runs as remote-key steps, every receive one kernel reading the
 * senders' buffers over IPC. C1_REGISTERED=1 takes the send buffer from the
 * group's registered memory (device, or shared memory with
 * UCX_BUILTIN_SHM_ZCOPY_THRESH), exposed in place.
 * C1_PPN=p [C1_SOCKET=s] places the members on hosts of p consecutive
 * members (sockets of s) through ucg_builtin_lgroup_create_ex; the planner
 * knobs come from the environment (UCX_BUILTIN_TREE_RADIX, ...).
 *
 * The "MPI library" behind reduce_cb_f is a plain C loop with MPI's operand
 * order (inoutvec[i] = invec[i] + inoutvec[i]); inputs are exact integers so
 * its NaN handling never matters, nor does the tree plan's arrival order
 * (non-power-of-two worlds). The result of every member is checked bit
 * for bit against the oracle's simulation of the reference plan
 * (oracle/combine_ref.c, test infrastructure). Member 0 prints one JSON line.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ucg_builtin_ops.h"
#include "combine_ref.h"

static int mini_reduce(void *op, char *src, char *dst, unsigned count, void *dt)
{
    const float *s = (const float*)src;
    float *d = (float*)dst;
    unsigned i;
    (void)op;
    (void)dt;
    for (i = 0; i < count; i++) {
        d[i] = s[i] + d[i];
    }
    return 0;
}

static int is_sum(void *op) { (void)op; return 1; }
static int no(void *op) { (void)op; return 0; }
static int yes(void *op) { (void)op; return 1; }
static int convert(void *dt, uintptr_t *u) { (void)dt; *u = 4u << 3; return 0; }
static int is_int(void *dt, int *s) { (void)dt; *s = 0; return 0; }
static int is_fp(void *dt) { (void)dt; return 1; }

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const char *name = argc > 1 ? argv[1] : "ucg_c1";
    int iters        = argc > 2 ? atoi(argv[2]) : 10000;
    size_t max_short = argc > 3 ? (size_t)atol(argv[3]) : 256;
    int count        = argc > 4 ? atoi(argv[4]) : 1024;
    unsigned rank    = (unsigned)atoi(getenv("RANK") ? getenv("RANK") : "0");
    unsigned world   = (unsigned)atoi(getenv("WORLD_SIZE") ? getenv("WORLD_SIZE") : "1");
    ucg_builtin_reduce_params_t rp = {mini_reduce, is_sum, no, yes, convert,
                                      is_int, is_fp};
    ucg_builtin_combine_config_t cfg = {0, 1u << 20, 8u << 20, 4, -1, 0, 0, NULL};
    ucg_builtin_combine_t *cmb;
    ucg_builtin_shm_iface_t *iface;
    ucg_builtin_lgroup_t *g;
    ucg_builtin_lcoll_t *c;
    float **inputs, *out, *want;
    unsigned r;
    int i, ok, placed;
    uint8_t dist[UCG_BUILTIN_OPS_MAX_MEMBERS];
    ucg_builtin_lgroup_params_t gp = {NULL, 0, 0, 0, 0};
    double t0, us;
    const int devbufs = getenv("C1_DEVICE_BUFFERS") != NULL;
    ucg_builtin_dev_ctx_t *dev = NULL;
    void *dsend = NULL, *drecv = NULL, *inputs_reg = NULL;

    /* the configuration read the way UCX reads it (UCX_BUILTIN_DEV_*) */
    ucg_builtin_combine_config_read(&cfg);
    if (!getenv("C1_DEVICE_STAGING") && !getenv("C1_DEVICE_BUFFERS")) {
        cfg.dev_enable = 0;       /* host buffers: every combine on reduce_cb_f */
    }
    if (getenv("C1_DEVICE_STAGING")) {
        /* every step staged on the GPU, forced on for any size */
        cfg.dev_enable    = 2;
        cfg.dev_min_bytes = 0;
    }
    if (devbufs) {
        int n = ucg_builtin_dev_device_count();
        cfg.dev_enable = 1;
        cfg.device     = n > 0 ? (int)(rank % (unsigned)n) : 0;
    }
    {
        const char *pp = getenv("C1_PPN"), *ps = getenv("C1_SOCKET");
        unsigned ppn = pp ? (unsigned)atoi(pp) : world, sock = ps ? (unsigned)atoi(ps) : 0;
        for (r = 0; r < world && r < UCG_BUILTIN_OPS_MAX_MEMBERS; r++) {
            dist[r] = (r == rank) ? UCG_BUILTIN_DISTANCE_SELF :
                      (r / ppn != rank / ppn) ? UCG_BUILTIN_DISTANCE_NET :
                      (sock && r / sock != rank / sock) ? UCG_BUILTIN_DISTANCE_HOST :
                      sock ? UCG_BUILTIN_DISTANCE_SOCKET : UCG_BUILTIN_DISTANCE_HOST;
        }
        placed = (pp != NULL || ps != NULL);
    }
    gp.distance = placed ? dist : NULL;
    if (ucg_builtin_combine_create(&rp, &cfg, &cmb) != UCS_OK ||
        ucg_builtin_shm_iface_open(name, world, rank, max_short, 64, &iface) != UCS_OK ||
        ucg_builtin_lgroup_create_ex(iface, 1, world, rank, cmb, &gp, &g) != UCS_OK) {
        fprintf(stderr, "rank %u: set-up failed\n", rank);
        return 1;
    }
    inputs = calloc(world, sizeof(*inputs));
    for (r = 0; r < world; r++) {
        inputs[r] = malloc(count * sizeof(float));
        ucg_oracle_fill(ORA_F32, ORA_DIST_EXACT, 0xC1000 + r, inputs[r], count);
    }
    out  = calloc(count, sizeof(float));
    want = calloc(count, sizeof(float));
    if ((world & (world - 1)) == 0 && !getenv("UCX_BUILTIN_ALLREDUCE_PLAN") && !placed) {
        ucg_oracle_reduce_multi(ORA_SUM, ORA_F32, want, (const void *const*)inputs,
                                world, rank, count);
    } else {   /* tree or multi-level plans; exact inputs make the
                * association (and arrival order) irrelevant */
        ucg_oracle_tree_reduce(ORA_SUM, ORA_F32, want, (const void *const*)inputs,
                               world, 0, NULL, count);
    }
    if (getenv("C1_REGISTERED")) {
        dev = devbufs ? ucg_builtin_combine_dev_ctx(cmb) : NULL;
        dsend = ucg_builtin_lgroup_mem_alloc(g, count * sizeof(float), devbufs);
        if (dsend == NULL) {
            fprintf(stderr, "rank %u: no registered memory\n", rank);
            return 1;
        }
        if (devbufs) {
            ucg_builtin_dev_memcpy(dev, dsend, inputs[rank], count * sizeof(float));
        } else {
            memcpy(dsend, inputs[rank], count * sizeof(float));
        }
        inputs_reg = dsend;
        dsend = NULL;
    }
    if (devbufs) {
        dev = ucg_builtin_combine_dev_ctx(cmb);
        dsend = dev ? ucg_builtin_dev_malloc(dev, count * sizeof(float)) : NULL;
        drecv = dev ? ucg_builtin_dev_malloc(dev, count * sizeof(float)) : NULL;
        if (dsend == NULL || drecv == NULL ||
            ucg_builtin_dev_memcpy(dev, dsend, inputs[rank], count * sizeof(float)) != UCS_OK) {
            fprintf(stderr, "rank %u: no device buffers\n", rank);
            return 1;
        }
    }
    if (ucg_builtin_lcoll_allreduce(g, inputs_reg ? inputs_reg :
                                       devbufs ? dsend : (void*)inputs[rank],
                                    devbufs ? drecv : (void*)out, count, (void*)1,
                                    (void*)1, &c) != UCS_OK) {
        fprintf(stderr, "rank %u: allreduce create failed\n", rank);
        return 1;
    }
    for (i = 0; i < (count > 65536 ? 2 : 100); i++) {        /* warm-up */
        if (ucg_builtin_lcoll_start(c) == UCS_INPROGRESS) {
            ucg_builtin_lcoll_wait(c);
        }
    }
    ucg_builtin_shm_barrier(iface);
    t0 = now_s();
    for (i = 0; i < iters; i++) {
        ucs_status_t st = ucg_builtin_lcoll_start(c);
        if (st == UCS_INPROGRESS) {
            st = ucg_builtin_lcoll_wait(c);
        }
        if (st != UCS_OK) {
            fprintf(stderr, "rank %u: allreduce failed %d\n", rank, st);
            return 1;
        }
    }
    us = (now_s() - t0) / iters * 1e6;
    if (devbufs && ucg_builtin_dev_memcpy(dev, out, drecv, count * sizeof(float)) != UCS_OK) {
        fprintf(stderr, "rank %u: download failed\n", rank);
        return 1;
    }
    ok = memcmp(out, want, count * sizeof(float)) == 0;
    ucg_builtin_shm_barrier(iface);
    if (rank == 0) {
        uint64_t st[4], cs[6];
        ucg_builtin_lgroup_stats(g, st);
        ucg_builtin_combine_stats(cmb, cs);
        printf("{\"config\": \"C1: %u-rank loopback allreduce, %d fp32 SUM%s\", "
               "\"ranks\": %u, \"bytes\": %zu, \"max_short\": %zu, "
               "\"latency_us\": %.3f, \"iters\": %d, \"bit_exact\": %s, "
               "\"messages_sent\": %llu, \"stashed\": %llu, "
               "\"host_combines\": %llu, \"device_combines\": %llu, "
               "\"device_staged_steps\": %llu}\n",
               world, count, devbufs ? ", device buffers" : "", world,
               count * sizeof(float), max_short, us, iters,
               ok ? "true" : "false", (unsigned long long)st[0],
               (unsigned long long)st[2], (unsigned long long)cs[0],
               (unsigned long long)cs[2], (unsigned long long)cs[4]);
    }
    ucg_builtin_lcoll_destroy(c);
    if (inputs_reg) {
        ucg_builtin_lgroup_mem_free(g, inputs_reg);
    }
    ucg_builtin_lgroup_destroy(g);
    if (devbufs) {
        ucg_builtin_dev_free(dev, dsend);
        ucg_builtin_dev_free(dev, drecv);
    }
    ucg_builtin_shm_iface_close(iface);
    ucg_builtin_combine_destroy(cmb);
    for (r = 0; r < world; r++) {
        free(inputs[r]);
    }
    free(inputs);
    free(out);
    free(want);
    return ok ? 0 : 3;
}

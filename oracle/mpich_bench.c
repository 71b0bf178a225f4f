/*
 * mpich_bench.c - TEST INFRASTRUCTURE (CPU baseline): the combine the
 * reference itself runs. builtin/ops calls the MPI library's reduction op
 * through reduce_cb_f (builtin/ops/builtin_comp_step.inl:96-102); in this
 * image that library is MPICH 3.3.2 (/opt/conda), whose MPI_Reduce_local(in =
 * src, inout = dst) is exactly the reduce_cb_f contract. This
 * times it on the host cores, fp32 SUM, the reference's two call shapes:
 *   whole   one call over the whole buffer (ucg_builtin_mpi_reduce_single)
 *   frag    one call per AM fragment ((max_short - 8) rounded to whole
 *           elements, ucg_builtin_mpi_reduce_fragment)
 * One thread (UCG combines on its progress thread). Inputs from the oracle's
 * generator; the result is checked against the oracle restatement.
 *
 *   mpich_bench [count] [budget_seconds] [max_short]
 *
 * Prints one JSON line (GiB/s on the 3N-byte basis).
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "combine_ref.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

static double whole(const float *src, float *dst, size_t n)
{
    double t0 = now_s();
    MPI_Reduce_local((void*)src, dst, (int)n, MPI_FLOAT, MPI_SUM);
    return now_s() - t0;
}

static double fragmented(const float *src, float *dst, size_t n, size_t frag_elems)
{
    double t0 = now_s();
    size_t i;
    for (i = 0; i < n; i += frag_elems) {
        size_t c = n - i < frag_elems ? n - i : frag_elems;
        MPI_Reduce_local((void*)(src + i), dst + i, (int)c, MPI_FLOAT, MPI_SUM);
    }
    return now_s() - t0;
}

int main(int argc, char **argv)
{
    size_t n         = argc > 1 ? (size_t)atol(argv[1]) : ((size_t)1 << 26);
    double budget    = argc > 2 ? atof(argv[2]) : 5.0;
    size_t max_short = argc > 3 ? (size_t)atol(argv[3]) : 8192;
    size_t frag      = ucg_oracle_frag_length(max_short, 4) / 4;
    float *src = malloc(n * 4), *dst = malloc(n * 4), *want = malloc(n * 4);
    double *t = NULL, first, gib = 3.0 * n * 4 / 1073741824.0;
    int reps, i, ok;

    if (src == NULL || dst == NULL || want == NULL || frag == 0) {
        fprintf(stderr, "mpich_bench: bad arguments or out of memory\n");
        return 1;
    }
    MPI_Init(&argc, &argv);
    ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 0x5EED0000, src, n);
    ucg_oracle_fill(ORA_F32, ORA_DIST_ROUND, 0x5EED0001, dst, n);
    memcpy(want, dst, n * 4);
    ucg_oracle_reduce(ORA_SUM, ORA_F32, src, want, n);
    first = whole(src, dst, n);
    ok = memcmp(dst, want, n * 4) == 0;

    reps = (int)(budget / 2 / (first > 1e-6 ? first : 1e-6));
    reps = reps < 5 ? 5 : (reps > 1000 ? 1000 : reps);
    t = malloc(sizeof(double) * reps);
    for (i = 0; i < reps; i++) {
        t[i] = whole(src, dst, n);
    }
    qsort(t, reps, sizeof(double), cmp_d);
    {
        double best_w = t[0], med_w = t[reps / 2], best_f, med_f;
        for (i = 0; i < reps; i++) {
            t[i] = fragmented(src, dst, n, frag);
        }
        qsort(t, reps, sizeof(double), cmp_d);
        best_f = t[0];
        med_f  = t[reps / 2];
#ifndef MPICH_VERSION
#define MPICH_VERSION "?"
#endif
        printf("{\"library\": \"MPICH %s MPI_Reduce_local\", \"count\": %zu, "
               "\"reps\": %d, \"whole_gibs\": %.3f, \"whole_best_gibs\": %.3f, "
               "\"fragment_bytes\": %zu, \"fragmented_gibs\": %.3f, "
               "\"fragmented_best_gibs\": %.3f, \"threads\": 1, \"bit_exact_vs_oracle\": %s}\n",
               MPICH_VERSION, n, reps, gib / med_w, gib / best_w,
               frag * 4, gib / med_f, gib / best_f, ok ? "true" : "false");
    }
    MPI_Finalize();
    free(t);
    free(src);
    free(dst);
    free(want);
    return ok ? 0 : 3;
}

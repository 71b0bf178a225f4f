/*
 * gen_golden.c - produce golden vectors for the combine path from MPICH.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/combine_ref.h). Built and run in the
 * dev container only, where MPICH 3.3.2 lives at /opt/conda:
 *     make -C oracle golden
 *
 * For every MPI integer type, MPI_FLOAT and MPI_DOUBLE it writes
 * tests/golden/raw_<dt>.bin holding the inputs (all special-value pairs, then
 * UCG_GOLD_NRAND "round" elements, then UCG_GOLD_NRAND "exact" elements) and,
 * for every MPI op, the output of MPI_Reduce_local(in=src, inout=dst) - the
 * exact call shape of reduce_cb_f(op, src, dst, count, dtype) used by
 * ucg_builtin_mpi_reduce, builtin/ops/builtin_comp_step.inl:96-102.
 * tests/golden/make_golden.py turns the raw files into .npz fixtures and adds
 * fp16 (numpy) and bf16 (torch) vectors.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "combine_ref.h"

#define UCG_GOLD_NRAND 259

static MPI_Datatype mpi_dt(int dt)
{
    switch (dt) {
    case ORA_I8:  return MPI_INT8_T;
    case ORA_U8:  return MPI_UINT8_T;
    case ORA_I16: return MPI_INT16_T;
    case ORA_U16: return MPI_UINT16_T;
    case ORA_I32: return MPI_INT32_T;
    case ORA_U32: return MPI_UINT32_T;
    case ORA_I64: return MPI_INT64_T;
    case ORA_U64: return MPI_UINT64_T;
    case ORA_F32: return MPI_FLOAT;
    case ORA_F64: return MPI_DOUBLE;
    default:      return MPI_DATATYPE_NULL;
    }
}

static MPI_Op mpi_op(int op)
{
    static const MPI_Op ops[ORA_OP_LAST] = {
        MPI_SUM, MPI_PROD, MPI_MAX, MPI_MIN, MPI_LAND, MPI_LOR, MPI_LXOR,
        MPI_BAND, MPI_BOR, MPI_BXOR};
    return ops[op];
}

static void store(void *buf, size_t sz, size_t i, uint64_t v)
{
    switch (sz) {
    case 1: ((uint8_t*)buf)[i]  = (uint8_t)v;  break;
    case 2: ((uint16_t*)buf)[i] = (uint16_t)v; break;
    case 4: ((uint32_t*)buf)[i] = (uint32_t)v; break;
    default: ((uint64_t*)buf)[i] = v;          break;
    }
}

int main(int argc, char **argv)
{
    const char *outdir = (argc > 1) ? argv[1] : "tests/golden";
    int dts[] = {ORA_I8, ORA_U8, ORA_I16, ORA_U16, ORA_I32, ORA_U32, ORA_I64,
                 ORA_U64, ORA_F32, ORA_F64};
    unsigned k;

    MPI_Init(&argc, &argv);
    for (k = 0; k < sizeof(dts) / sizeof(dts[0]); k++) {
        int dt = dts[k], op;
        size_t sz = ucg_oracle_dtype_size(dt), i, j;
        uint64_t tab[32];
        size_t ns = ucg_oracle_special_table(dt, tab, 32);
        size_t npair = ns * ns;
        size_t n = npair + 2 * UCG_GOLD_NRAND;
        char *src = malloc(n * sz), *dst = malloc(n * sz), *out = malloc(n * sz);
        char path[512];
        FILE *f;

        for (i = 0; i < ns; i++) {
            for (j = 0; j < ns; j++) {
                store(src, sz, i * ns + j, tab[i]);
                store(dst, sz, i * ns + j, tab[j]);
            }
        }
        ucg_oracle_fill(dt, ORA_DIST_ROUND, 0x5eed0000u + 4 * dt + 0,
                        src + npair * sz, UCG_GOLD_NRAND);
        ucg_oracle_fill(dt, ORA_DIST_ROUND, 0x5eed0000u + 4 * dt + 1,
                        dst + npair * sz, UCG_GOLD_NRAND);
        ucg_oracle_fill(dt, ORA_DIST_EXACT, 0x5eed0000u + 4 * dt + 2,
                        src + (npair + UCG_GOLD_NRAND) * sz, UCG_GOLD_NRAND);
        ucg_oracle_fill(dt, ORA_DIST_EXACT, 0x5eed0000u + 4 * dt + 3,
                        dst + (npair + UCG_GOLD_NRAND) * sz, UCG_GOLD_NRAND);

        snprintf(path, sizeof(path), "%s/raw_%d.bin", outdir, dt);
        f = fopen(path, "wb");
        if (!f) {
            perror(path);
            return 1;
        }
        uint32_t hdr[4] = {0x55434731u /* "UCG1" */, (uint32_t)dt, (uint32_t)n,
                           (uint32_t)ORA_OP_LAST};
        fwrite(hdr, sizeof(hdr), 1, f);
        fwrite(src, sz, n, f);
        fwrite(dst, sz, n, f);
        for (op = 0; op < ORA_OP_LAST; op++) {
            uint32_t ok = (uint32_t)ucg_oracle_is_supported(dt, op);
            memcpy(out, dst, n * sz);
            if (ok) {
                MPI_Reduce_local(src, out, (int)n, mpi_dt(dt), mpi_op(op));
            }
            fwrite(&ok, sizeof(ok), 1, f);
            fwrite(out, sz, n, f);
        }
        fclose(f);
        free(src);
        free(dst);
        free(out);
    }
    MPI_Finalize();
    return 0;
}

"""Pack golden vectors for the combine path into tests/golden/golden_<dt>.npz.

Run in the dev container (needs MPICH at /opt/conda, numpy and torch):
    make -C oracle golden
which first runs oracle/_build/gen_golden (MPICH 3.3.2 MPI_Reduce_local ->
raw_<dt>.bin for the integer types, fp32 and fp64) and then this script.

Sources of truth per dtype (see README.md next to this file):
  int8..uint64, float32, float64 : MPICH 3.3.2 MPI_Reduce_local(src, dst)
  float16                        : numpy 2.2 float16 arithmetic (SUM/PROD via
                                   np.add/np.multiply(src, dst)); MAX/MIN via
                                   numpy float16 comparisons + np.where
  bfloat16                       : torch CPU bfloat16 arithmetic for SUM/PROD
                                   (non-NaN results); MAX/MIN via float32
                                   comparisons + np.where
The inputs of every file are the special-value pairs followed by 259 "round"
and 259 "exact" elements of the counter-based generator (oracle.fill).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import oracle  # noqa: E402

NRAND = 259
OPS = oracle.OPS


def inputs(dt):
    dti = oracle.dt_index(dt)
    st = oracle.storage(dt)
    tab = np.array(oracle.special_table(dt), dtype=np.uint64)
    ns = len(tab)
    bits_t = oracle.NP_BITS[np.dtype(st).itemsize]
    s_sp = np.repeat(tab, ns).astype(bits_t).view(st)
    d_sp = np.tile(tab, ns).astype(bits_t).view(st)
    base = 0x5EED0000 + 4 * dti
    src = np.concatenate([s_sp, oracle.fill(dt, "round", base + 0, NRAND),
                          oracle.fill(dt, "exact", base + 2, NRAND)])
    dst = np.concatenate([d_sp, oracle.fill(dt, "round", base + 1, NRAND),
                          oracle.fill(dt, "exact", base + 3, NRAND)])
    return src, dst


def read_raw(dti):
    path = os.path.join(HERE, f"raw_{dti}.bin")
    with open(path, "rb") as f:
        hdr = np.frombuffer(f.read(16), dtype=np.uint32)
        assert hdr[0] == 0x55434731 and hdr[1] == dti
        n, nops = int(hdr[2]), int(hdr[3])
        st = oracle.storage(dti)
        sz = np.dtype(st).itemsize
        src = np.frombuffer(f.read(n * sz), dtype=st).copy()
        dst = np.frombuffer(f.read(n * sz), dtype=st).copy()
        outs, sup = [], []
        for _ in range(nops):
            ok = np.frombuffer(f.read(4), dtype=np.uint32)[0]
            outs.append(np.frombuffer(f.read(n * sz), dtype=st).copy())
            sup.append(bool(ok))
    os.remove(path)
    return src, dst, np.stack(outs), np.array(sup)


def f16_outputs(src, dst):
    outs, sup = [], []
    with np.errstate(all="ignore"):
        for op in OPS:
            if op == "sum":
                o = np.add(src, dst)      # MPI: invec (op) inoutvec
            elif op == "prod":
                o = np.multiply(src, dst)
            elif op == "max":
                o = np.where(dst > src, dst, src)
            elif op == "min":
                o = np.where(dst < src, dst, src)
            else:
                outs.append(dst.copy())
                sup.append(False)
                continue
            outs.append(o.astype(np.float16))
            sup.append(True)
    return np.stack(outs), np.array(sup)


def bf16_outputs(src, dst):
    import torch
    s32 = (src.astype(np.uint32) << 16).view(np.float32)
    d32 = (dst.astype(np.uint32) << 16).view(np.float32)
    ts = torch.from_numpy(src.view(np.int16).copy()).view(torch.bfloat16)
    td = torch.from_numpy(dst.view(np.int16).copy()).view(torch.bfloat16)
    outs, sup = [], []
    for op in OPS:
        if op in ("sum", "prod"):
            t = (ts + td) if op == "sum" else (ts * td)
            o = t.view(torch.int16).numpy().view(np.uint16).copy()
            # NaN results: torch's scalar and vector paths disagree
            # (0x7FC0 vs 0xFFFF), so NaN bits are restated by the oracle rule
            nan = np.isnan((o.astype(np.uint32) << 16).view(np.float32))
            ref = oracle.reduce(op, "bfloat16", src, dst)
            o[nan] = ref[nan]
        elif op == "max":
            o = np.where(d32 > s32, dst, src)
        elif op == "min":
            o = np.where(d32 < s32, dst, src)
        else:
            outs.append(dst.copy())
            sup.append(False)
            continue
        outs.append(o.astype(np.uint16))
        sup.append(True)
    return np.stack(outs), np.array(sup)


def main():
    for dt in oracle.DTYPES:
        dti = oracle.dt_index(dt)
        if dt == "float16":
            src, dst = inputs(dt)
            out, sup = f16_outputs(src, dst)
            source = "numpy-" + np.__version__
        elif dt == "bfloat16":
            import torch
            src, dst = inputs(dt)
            out, sup = bf16_outputs(src, dst)
            source = "torch-" + torch.__version__.split("+")[0]
        else:
            src, dst, out, sup = read_raw(dti)
            s2, d2 = inputs(dt)
            assert (oracle.bits(s2) == oracle.bits(src)).all()
            assert (oracle.bits(d2) == oracle.bits(dst)).all()
            source = "mpich-3.3.2"
        np.savez_compressed(os.path.join(HERE, f"golden_{dt}.npz"), src=src,
                            dst=dst, out=out, supported=sup,
                            source=np.array(source))
        print(f"golden_{dt}.npz: n={src.size} ops={int(sup.sum())} ({source})")


if __name__ == "__main__":
    main()

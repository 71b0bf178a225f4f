"""Do the two operands of the combine alias in HBM's channel/bank map? For P
separately allocated operand pairs (256 MiB + 64 KiB each), time the headline
combine (2^26 fp32 SUM) with src moved k x 4 KiB against dst, k = 0..15
(16-B aligned: the same kernel), interleaved over rounds. If the slow pairs
are slow at k = 0 only, the relative placement of src and dst decides, and a
4 KiB stagger between operands is the fix.

    python scripts/alias_probe.py OUT.json [pairs=6] [rounds=2] [--joint]

--joint: each pair is ONE allocation (src at 0, dst 256 MiB + k x 4 KiB after
it): the relative offset inside an arena, where it is also the physical one
as far as the allocation is physically contiguous.
"""
import json
import sys

sys.path.insert(0, ".")

N = 1 << 26
PAD = 64 << 10


def main():
    import xucg_amd
    out = sys.argv[1]
    npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    ctx = xucg_amd.DevContext(device=0)
    joint = "--joint" in sys.argv
    if joint:
        arenas = [ctx.alloc(2 * N * 4 + PAD) for _ in range(npairs)]
        pairs = [(a, a) for a in arenas]
        for a in arenas:
            ctx.fill("float32", "round", 11, a, (2 * N * 4 + PAD) // 4)
    else:
        pairs = [(ctx.alloc(N * 4 + PAD), ctx.alloc(N * 4 + PAD)) for _ in range(npairs)]
        for s, d in pairs:
            ctx.fill("float32", "round", 11, s, (N * 4 + PAD) // 4)
            ctx.fill("float32", "round", 12, d, N)
    ctx.sync()
    res = [[[] for _ in range(16)] for _ in pairs]
    for _ in range(rounds):
        for j, (s, d) in enumerate(pairs):
            for k in range(16):
                if joint:
                    src, dst = s.ptr, s.ptr + N * 4 + k * 4096
                else:
                    src, dst = s.ptr + k * 4096, d.ptr
                ctx.profile_reduce("sum", "float32", dst, src, N, 5)
                us = sorted(ctx.profile_reduce("sum", "float32", dst, src, N, 20)
                            for _ in range(3))[1]
                res[j][k].append(round(3 * N * 4 / (us * 1e-6) / 8e12, 4))
    med = [[sorted(v)[len(v) // 2] for v in row] for row in res]
    for j, row in enumerate(med):
        print(f"pair {j}: " + " ".join(f"{x:.3f}" for x in row), flush=True)
    with open(out, "w") as f:
        json.dump({"frac_by_pair_by_offset_4k": med, "joint": joint, "rounds": rounds,
                   "ptrs": [[hex(s.ptr), hex(d.ptr)] for s, d in pairs]}, f, indent=1)
    for b in ({id(x): x for p in pairs for x in p}).values():
        b.free()
    ctx.close()


if __name__ == "__main__":
    main()

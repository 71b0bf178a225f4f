"""Is the headline combine's slow state a property of the buffers or of the
time? One process, the 2^26 fp32 SUM combine of bench.py on differently
placed operand pairs, interleaved over several rounds (HIP events, median of
5 batches of 50 launches after 10 warm ones; 1 GiB pairs: batches of 20).

    python scripts/place_probe.py OUT.json [rounds] [--torch]

gib_src+Xk: the 1 GiB pair's first 256 MiB with src moved X KiB against dst
(aliasing of the two operands in the HBM channel/bank map).

Pairs: `first` (allocated first, as bench.py's), `gib` (a 1 GiB pair, the
north-star shape), `win0` / `win512` (256 MiB windows of the 1 GiB pair at 0
and 512 MiB), `joint` (src and dst in one 512 MiB allocation), `later` (a
256 MiB pair allocated after all the others). --torch initialises torch's
device context first, as bench.py does. If `first` stays slow while `gib` and
the windows stay fast across rounds, placement decides; if all move together,
time does."""
import json
import sys
import time

N = 1 << 26
NB = 1 << 28


def main():
    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 6
    if "--torch" in sys.argv:
        import torch
        torch.zeros(1, device="cuda").sum().item()
    sys.path.insert(0, ".")
    import xucg_amd
    ctx = xucg_amd.DevContext(device=0)
    bufs = []

    def alloc(nbytes):
        b = ctx.alloc(nbytes)
        bufs.append(b)
        return b

    s_first, d_first = alloc(N * 4), alloc(N * 4)
    s_gib, d_gib = alloc(NB * 4), alloc(NB * 4)
    joint = alloc(2 * N * 4)
    s_later, d_later = alloc(N * 4), alloc(N * 4)
    pairs = {
        "first": (d_first, s_first, N),
        "gib": (d_gib, s_gib, NB),
        "win0": (d_gib, s_gib, N),
        "win512": (d_gib.offset(512 << 20), s_gib.offset(512 << 20), N),
        "joint": (joint.offset(N * 4), joint, N),
        "later": (d_later, s_later, N),
    }
    # the same 1 GiB pair with src moved against dst by a few bytes to MiB
    # inside its allocation (16-B aligned: the same kernel): if the slow pairs
    # are slow because src and dst alias in HBM's channel/bank map, some
    # offsets recover the rate
    for off in (4 << 10, 64 << 10, 1 << 20, (2 << 20) + (4 << 10), (16 << 20) + (64 << 10)):
        pairs[f"gib_src+{off >> 10}k"] = (d_gib, s_gib.offset(off), N)
    for name, (d, s, n) in pairs.items():
        ctx.fill("float32", "round", 11, s, n)
        ctx.fill("float32", "round", 12, d, n)
    ctx.sync()
    res = {k: [] for k in pairs}
    ro = {k: [] for k in pairs}
    t0 = time.time()
    for r in range(rounds):
        for name, (d, s, n) in pairs.items():
            it = 20 if n == NB else 50
            ctx.profile_reduce("sum", "float32", d, s, n, 10)
            b = sorted(ctx.profile_reduce("sum", "float32", d, s, n, it) for _ in range(5))
            res[name].append(round(3 * n * 4 / (b[2] * 1e-6) / 8e12, 4))
            b = sorted(ctx.profile_stream(0, d, s, n * 4, it) for _ in range(3))
            ro[name].append(round(2 * n * 4 / (b[1] * 1e-6) / 8e12, 4))
        line = {"round": r, "t_s": round(time.time() - t0, 2),
                **{k: v[-1] for k, v in res.items()}}
        print(json.dumps(line), flush=True)
    with open(out, "w") as f:
        json.dump({"frac_of_8tbs": res, "read_only_frac": ro,
                   "torch_first": "--torch" in sys.argv}, f, indent=1)
    for b in bufs:
        b.free()


if __name__ == "__main__":
    main()

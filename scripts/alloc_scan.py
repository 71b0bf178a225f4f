"""Is HBM streaming speed a property of the allocation? One process
allocates a sequence of buffers (hipMalloc through the device shim) and times
a read-only stream over each one alone (its two halves read as the two
operands of the combine's geometry, ucg_builtin_dev_profile_stream kind 0),
in several interleaved rounds. A buffer that is slow in every round while its
neighbours are fast is slow by placement, not by time.

    python scripts/alloc_scan.py OUT.json [count=24] [mib=256] [rounds=3] [window_mib]

With window_mib, every allocation is scanned in windows of that size (is the
speed a property of the whole allocation or of regions inside it?).
"""
import json
import sys

sys.path.insert(0, ".")


def main():
    import xucg_amd
    out = sys.argv[1]
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    mib = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    ctx = xucg_amd.DevContext(device=0)
    nbytes = mib << 20
    bufs = [ctx.alloc(nbytes) for _ in range(count)]
    for b in bufs:
        ctx.fill("float32", "round", 5, b, nbytes // 4)
    ctx.sync()
    win = (int(sys.argv[5]) << 20) if len(sys.argv) > 5 else nbytes
    spans = [(b.ptr + off, win) for b in bufs for off in range(0, nbytes, win)]
    rates = [[] for _ in spans]
    for _ in range(rounds):
        for i, (p, w) in enumerate(spans):
            half = w // 2
            ctx.profile_stream(0, p + half, p, half, 5)
            us = sorted(ctx.profile_stream(0, p + half, p, half, 20) for _ in range(3))[1]
            rates[i].append(round(w / (us * 1e-6) / 8e12, 4))
    med = [sorted(r)[len(r) // 2] for r in rates]
    print(json.dumps({"mib": mib, "window_mib": win >> 20,
                      "read_only_frac_in_order": med}), flush=True)
    with open(out, "w") as f:
        json.dump({"mib": mib, "window_mib": win >> 20, "count": count, "rounds": rounds,
                   "frac": rates,
                   "median": med, "ptrs": [hex(b.ptr) for b in bufs]}, f, indent=1)
    for b in bufs:
        b.free()
    ctx.close()


if __name__ == "__main__":
    main()

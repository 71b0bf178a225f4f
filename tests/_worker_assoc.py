"""One member of a multi-process collective whose combine RECORDS the
association instead of computing a value.

    _worker_assoc.py <shm-name> <kind> <max_short> <count> [key=value ...]

kind: "allreduce" or "reduce"; keys: factor (RECURSIVE_FACTOR), ppn (members
per host, by-node layout), root (reduce).

The datatype is a contiguous 64-byte type the device path cannot classify,
so every combine goes to reduce_cb_f, which here writes the expression
"(" src dst ")" into dst: member r's input is the one-letter leaf
chr(ord('a') + r), and the result of the collective is the exact tree of
reduce_cb_f calls that produced it, operand roles included.

The expected trees are written below from the reference's text, not from
this repository's planner or from oracle/plans.py (a transliteration of the
same planner code): the accumulator starts as the member's own send buffer
(builtin_control.c:43-47); every incoming message is reduced as
dst = incoming (op) dst (builtin_comp_step.inl:96-102, 213-221); recursive
doubling/K-ing peers are base + ((my - base + size * i) % (size * factor))
with size starting at the members per host (builtin_recursive.c:140-169);
members of a host fan in to the host's lowest member first and get the
result back by fan-out (builtin_tree.c:262-351 with builtin_recursive.c:45-
56, 116-129, 172-186); a group that is not a power of the factor reduces
on the flat one-host tree at member 0 (builtin_recursive.c:78-88,
builtin.c:112-121). Messages from several peers of one step arrive in any
order, so those trees are checked up to the order of the peers."""
import ctypes
import hashlib
import os
import sys

import numpy as np

from xucg_amd import host, ops

ELEM = 64
DT_TRACE = 0x9000
OP_TRACE = 0x4000


class TraceMPI:
    """reduce_cb_f builds the expression tree of the reduction in dst."""

    def __init__(self):
        self.calls = 0
        self.too_long = 0

    def reduce_cb_f(self, op, src, dst, count, dtype):
        if dtype != DT_TRACE:
            return 1
        self.calls += 1
        s = (ctypes.c_char * (count * ELEM)).from_address(src).raw
        d = (ctypes.c_char * (count * ELEM)).from_address(dst)
        out = bytearray(count * ELEM)
        for i in range(count):
            a = s[i * ELEM:(i + 1) * ELEM].rstrip(b"\0")
            b = d.raw[i * ELEM:(i + 1) * ELEM].rstrip(b"\0")
            e = b"(" + a + b + b")"
            if len(e) > ELEM:
                self.too_long += 1
                return 1
            out[i * ELEM:i * ELEM + len(e)] = e
        ctypes.memmove(dst, bytes(out), count * ELEM)
        return 0

    def callbacks(self):
        return {"reduce_cb_f": self.reduce_cb_f,
                "is_sum_f": lambda op: op == OP_TRACE,
                "is_loc_expected_f": lambda op: False,
                "is_commutative_f": lambda op: True,
                "convert": lambda dt: ELEM << 3,            # contiguous, 64 B
                "is_integer_f": lambda dt: (False, False),
                "is_floating_point_f": lambda dt: False}


# ---- the expected trees, as predicates over parsed trees ------------------
def parse(s):
    """'(' S D ')' | leaf letter  ->  nested tuples (S, D) / str"""
    pos = 0

    def one():
        nonlocal pos
        if pos >= len(s):
            raise ValueError("truncated")
        c = s[pos]
        pos += 1
        if c != "(":
            return c
        a = one()
        b = one()
        if pos >= len(s) or s[pos] != ")":
            raise ValueError("unbalanced")
        pos += 1
        return (a, b)

    t = one()
    if pos != len(s):
        raise ValueError("trailing bytes")
    return t


def leaf(r):
    return chr(ord("a") + r)


def is_leaf(r):
    return lambda t: t == leaf(r)


def chain(inner_spec, incoming_specs):
    """an accumulator seeded with `inner` that received every one of
    `incoming` once, in any order: (m_k (... (m_1 inner)))"""
    def check(t, pending):
        if not pending:
            return inner_spec(t)
        if not isinstance(t, tuple):
            return False
        for k, spec in enumerate(pending):
            if spec(t[0]) and check(t[1], pending[:k] + pending[k + 1:]):
                return True
        return False
    return lambda t: check(t, list(incoming_specs))


def recursive_spec(my, n, factor, ppn):
    """builtin_recursive.c: fan-in inside the host (ppn > 1), then K-ing over
    the host masters with steps of size ppn, ppn*factor, ..."""
    def host_fanin(m):
        return chain(is_leaf(m), [is_leaf(c) for c in range(m + 1, m + ppn)])

    def acc(m, size):
        """member m's accumulator once the steps below `size` are done"""
        if size == ppn:
            return host_fanin(m) if ppn > 1 else is_leaf(m)
        prev = size // factor
        base = m - m % size
        peers = [base + (m - base + prev * i) % size for i in range(1, factor)]
        return chain(acc(m, prev), [acc(p, prev) for p in peers])

    master = my - my % ppn
    return acc(master, n)


def tree_spec(n, root):
    """the flat one-host fan-in at the root: its own data, then every other
    member's once"""
    return chain(is_leaf(root), [is_leaf(m) for m in range(n) if m != root])


def is_power(n, k):
    while n % k == 0 and n > 1:
        n //= k
    return n == 1


def expected(kind, n, my, factor, ppn, root):
    """the tree member `my` must hold, and its name. MPI_Reduce is the fan-in
    tree and MPI_Allreduce the recursive plan for a power-of-two group, the
    fan-in/fan-out tree otherwise (ucg_builtin_choose_topology, builtin.c:
    94-131); the recursive plan falls back to the one-host tree when the
    group is not a power of the factor (builtin_recursive.c:74-88)."""
    hosts = n // ppn
    host_fanin = lambda m: chain(is_leaf(m), [is_leaf(c) for c in range(m + 1, m + ppn)])
    if kind == "reduce":
        assert hosts == 1
        return tree_spec(n, root), f"flat fan-in at {root}"
    if bin(n).count("1") > 1 or (hosts == 1 and not is_power(n, factor)):
        # fan-in to member 0: its host's members, then the other hosts'
        # masters, each holding its own host's fan-in (inter-host radix 8)
        assert hosts <= 8
        spec = chain(host_fanin(0), [host_fanin(m) for m in range(ppn, n, ppn)])
        return spec, f"fan-in at 0 over {hosts} host(s) + fan-out"
    if hosts == 1:
        return recursive_spec(my, n, factor, 1), f"recursive factor {factor}"
    return recursive_spec(my, n, factor, ppn), f"host fan-in + recursive over {hosts} masters"


def main():
    name, kind, max_short, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    kv = dict(a.split("=") for a in sys.argv[5:])
    factor, ppn, root = int(kv.get("factor", 2)), int(kv.get("ppn", 0)), int(kv.get("root", 0))
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])

    mpi = TraceMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0),
                              op_classifier=lambda op: -1, dt_classifier=lambda dt: -1)
    iface = ops.ShmIface(name, world, rank, max_short=max_short)
    dist = ops.layout_distances(world, rank, ppn=ppn) if ppn else None
    group = ops.Group(iface, 11, world, rank, cmb, distance=dist, factor=factor)

    sbuf = np.zeros(count * ELEM, dtype=np.uint8)
    sbuf.reshape(count, ELEM)[:, 0] = ord(leaf(rank))
    rbuf = np.zeros_like(sbuf)
    if kind == "allreduce":
        coll = group.allreduce(sbuf, rbuf, count, DT_TRACE, OP_TRACE)
    else:
        coll = group.reduce(sbuf, rbuf if rank == root else None, count, DT_TRACE, OP_TRACE,
                            root=root)
    if coll.status != 0:
        print(f"rank {rank}: create status {coll.status}", flush=True)
        sys.exit(1)
    plan = coll.describe() if rank == 0 else ""
    rc = 0
    for rep in range(2):                     # the persistent op, started twice
        rbuf[:] = 0
        iface.barrier()
        st = coll.run()
        if st != 0:
            print(f"rank {rank}: status {st} (too long: {mpi.too_long})", flush=True)
            sys.exit(1)
        if kind == "reduce" and rank != root:
            continue
        rows = [bytes(r).rstrip(b"\0").decode() for r in rbuf.reshape(count, ELEM)]
        spec, what = expected(kind, world, rank, factor, ppn or world, root)
        # fragments arrive independently, so where a step has several peers
        # each element may hold its own order: every element is checked
        for i, got in enumerate(rows):
            try:
                ok = spec(parse(got))
            except ValueError as e:
                ok, got = False, f"{got}  <{e}>"
            if not ok:
                print(f"rank {rank}: ASSOCIATION MISMATCH ({what}) element {i}: {got}",
                      flush=True)
                rc = 1
                break
        # a member that got its result by fan-out holds its master's bits
        print(f"rank {rank}: rep {rep} result {rows[0]} rows "
              f"{hashlib.sha1(''.join(rows).encode()).hexdigest()[:16]}", flush=True)
    if plan:
        print(plan, flush=True)
    print(f"rank {rank}: reduce_cb_f calls {mpi.calls}", flush=True)
    coll.close()
    group.close()
    iface.close()
    cmb.close()
    if rc == 0:
        print(f"rank {rank}: ok", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()

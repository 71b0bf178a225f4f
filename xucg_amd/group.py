"""Multi-rank execution of the combine path: one process per GPU.

torch.distributed is the plumbing (RCCL over xGMI on the GPU box, gloo for
CPU tests); every combine runs through the C-ABI device shim. Four ways to
allreduce a buffer across 2^k members, all built on the same combine:

  recursive_doubling_allreduce  the reference plan itself
                                (builtin/plan/builtin_recursive.c:158-169):
                                at step k exchange the whole accumulator with
                                member my ^ 2^(k-1), then acc = incoming (op)
                                acc. Bit-exact with the reference.
  oneshot_reduce_scatter        every member owns a contiguous shard and reads
                                that shard from all members at once (peer
                                mapped, xGMI), evaluating the same per-element
                                association as the plan in registers
                                (ucg_builtin_dev_reduce_multi); followed by an
                                all-gather. Bit-exact with the plan's result
                                on the shard owner. Groups that are not a
                                power of two get the plan the reference takes
                                there, the tree fan-in at member 0
                                (ucg_builtin_dev_reduce_tree), so the one-shot
                                forms work for any size up to 16.
  recursive_halving_allreduce   reduce-scatter by recursive halving with the
                                plan's peer order (my ^ 1, my ^ 2, ...) then
                                all-gather by recursive doubling (SURVEY.md 8e,
                                config 5). Every element gets the plan's
                                association on the member that ends up owning
                                it, so the result equals the plan's bit for bit
                                (for a commutative op without NaN payload
                                choices, on every member); it moves
                                2 (N-1)/N x S per member instead of log2(N) x S.
  RCCL reduce_scatter + all_gather  the vendor baseline (ring association:
                                within the fp tolerance of SURVEY.md 8c only).
"""
import numpy as np

from . import _lib

SHARD_ALIGN_BYTES = 256


def shard_bounds(count, elem_size, world, rank, align_bytes=SHARD_ALIGN_BYTES):
    """[lo, hi) element range of `rank`'s shard: equal shards
    rounded down to `align_bytes`, the remainder to the last rank."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    align = align_bytes // elem_size if align_bytes % elem_size == 0 else 1
    per = (count // world) // align * align
    lo = per * rank
    hi = count if rank == world - 1 else per * (rank + 1)
    return lo, hi


def recursive_steps(world, factor=2):
    """Number of recursive steps, 0 when world is not a power of factor
    (builtin/plan/builtin_recursive.c:76-88)."""
    return _lib.host().ucg_builtin_recursive_steps(world, factor)


def recursive_peer(rank, step, factor=2, peer_idx=1):
    return _lib.host().ucg_builtin_recursive_peer(rank, step, factor, peer_idx)


def recursive_doubling_allreduce(acc, tmp, rank, world, combine, exchange):
    """The reference recursive-doubling plan.

    acc      this member's contribution on entry, the allreduce on exit
             (ucg_builtin_init_reduce seeds recv <- send, builtin_control.c:43-47)
    tmp      receive buffer of the same size
    combine  combine(dst=acc, src=tmp): dst = src (op) dst
    exchange exchange(send=acc, recv=tmp, peer): full-vector swap
    """
    if world == 1:
        return
    steps = recursive_steps(world)
    if steps == 0:
        raise ValueError("recursive doubling needs a power-of-two group "
                         "(builtin_recursive.c:78-88 returns UNSUPPORTED)")
    for step in range(1, steps + 1):
        peer = recursive_peer(rank, step)
        exchange(acc, tmp, peer)
        combine(acc, tmp)


def _halve(lo, hi, align):
    half = (hi - lo) // 2
    if half >= align:
        half -= half % align
    return lo + half


def recursive_halving_segments(count, world, align=1):
    """Element range [lo, hi) each member owns after the halving
    reduce-scatter (member bit k set: upper half at step k+1)."""
    steps = recursive_steps(world)
    out = []
    for rank in range(world):
        lo, hi = 0, count
        for k in range(steps):
            mid = _halve(lo, hi, align)
            lo, hi = (mid, hi) if rank & (1 << k) else (lo, mid)
        out.append((lo, hi))
    return out


def recursive_halving_allreduce(acc, tmp, rank, world, combine, exchange, count,
                                elem_size, align_bytes=SHARD_ALIGN_BYTES):
    """Recursive halving reduce-scatter + recursive doubling all-gather.

    acc, tmp  1-D tensors holding `count` elements of `elem_size` bytes (any
              torch dtype whose size divides elem_size)
    combine   combine(dst, src, n): dst = src (op) dst over n elements
    exchange  exchange(send, recv, peer): paired send/receive (lengths may
              differ by the odd element of a split)
    """
    if world == 1:
        return
    steps = recursive_steps(world)
    if steps == 0:
        raise ValueError("recursive halving needs a power-of-two group")
    per = elem_size // acc.element_size()
    align = max(1, align_bytes // elem_size) if align_bytes % elem_size == 0 else 1

    def seg(t, lo, hi):
        return t.narrow(0, lo * per, (hi - lo) * per)

    lo, hi = 0, count
    ranges = []
    for k in range(steps):                      # peers my^1, my^2, my^4, ...
        peer = rank ^ (1 << k)
        mid = _halve(lo, hi, align)
        keep, give = ((mid, hi), (lo, mid)) if rank & (1 << k) else ((lo, mid), (mid, hi))
        exchange(seg(acc, *give), seg(tmp, *keep), peer)
        combine(seg(acc, *keep), seg(tmp, *keep), keep[1] - keep[0])
        ranges.append((lo, hi))
        lo, hi = keep
    for k in reversed(range(steps)):            # all-gather: WRITE into acc
        peer = rank ^ (1 << k)
        plo, phi = ranges[k]
        theirs = (plo, lo) if lo > plo else (hi, phi)
        exchange(seg(acc, lo, hi), seg(acc, *theirs), peer)
        lo, hi = plo, phi


def torch_exchange(dist, group=None):
    """exchange() over torch.distributed point-to-point (RCCL or gloo)."""
    def exchange(send, recv, peer):
        ops = [dist.P2POp(dist.isend, send, peer, group),
               dist.P2POp(dist.irecv, recv, peer, group)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    return exchange


class PeerBuffers:
    """Every member's buffer mapped into this process (IPC over xGMI).

    ptrs[r] is a device pointer to member r's buffer (the local one for
    r == rank). Collective: every member must construct it together, and
    close it together; close() ends with a barrier, after which each member
    may free its buffer. A key names the buffer's physical allocation
    (ucg_builtin_dev_ipc_export): memory from the shim's shareable allocator
    (ctx.alloc(..., shareable=True), or any tensor after
    xucg_amd.use_shareable_torch_memory()) is mapped by its file descriptor,
    other memory by hipIpc, checked against the runtime's buffer id; a freed
    buffer's keys are refused. Memory from torch's own caching
    allocator recycles addresses, which this platform can serve through stale
    translations, so bench.py keeps such exported tensors
    allocated until its phases end."""

    def __init__(self, ctx, local_ptr, rank, world, dist, group=None):
        self.ctx = ctx
        self.rank = rank
        self._dist, self._group = dist, group
        self.ptrs = []
        self._imported = []
        # every member takes part in every collective below whatever fails
        # locally, and all members agree on the outcome: a failure raises on
        # all of them instead of leaving the others waiting
        err = None
        try:
            blob = ctx.ipc_export(local_ptr)
        except Exception as e:  # noqa: BLE001 - reported after agreement
            blob, err = None, e
        blobs = [None] * world
        dist.all_gather_object(blobs, blob, group=group)
        self.blobs = blobs          # the keys as exchanged (diagnostics)
        if err is None and any(b is None for b in blobs):
            err = RuntimeError("a peer failed to export its buffer")
        if err is None:
            try:
                for r, b in enumerate(blobs):
                    if r == rank:
                        self.ptrs.append(local_ptr)
                    else:
                        p = ctx.ipc_import(b)
                        self._imported.append(p)
                        self.ptrs.append(p)
            except Exception as e:  # noqa: BLE001
                err = e
        ok = [err is None]
        oks = [None] * world
        dist.all_gather_object(oks, ok, group=group)
        if err is None and not all(o[0] for o in oks):
            err = RuntimeError("a peer failed to map the group's buffers")
        if err is not None:
            self.close()
            raise RuntimeError(f"PeerBuffers: {err}")

    def close(self):
        """Release the peer mappings, then wait for every member to have done
        the same: after close() returns each member may free its buffer."""
        if self._dist is None:
            return
        err = None
        for p in self._imported:
            try:
                self.ctx.ipc_release(p)
            except Exception as e:  # noqa: BLE001 - after the barrier
                err = err or e
        self._imported = []
        dist, self._dist = self._dist, None
        dist.barrier(group=self._group)
        if err is not None:
            raise err


def is_pow2(n):
    return n > 0 and n & (n - 1) == 0


def _combine_shard(ctx, op, dt, out_ptr, srcs, rank, world, n):
    """One member's shard of a one-shot reduce-scatter, srcs in member order:
    the recursive-doubling plan's association V(rank, log2 N) for 2^k members
    (builtin_recursive.c:158-169), and for any other group size the plan the
    reference takes there - the tree fan-in at member 0 with the children
    arriving in ascending order (builtin.c:112-121, builtin_tree.c:262-380).
    Either way every member's shard is bit-identical to what that plan leaves
    in every member's buffer."""
    if is_pow2(world):
        _lib.check(ctx.reduce_multi(op, dt, out_ptr, srcs, rank, n),
                   "ucg_builtin_dev_reduce_multi")
    else:
        _lib.check(ctx.reduce_tree(op, dt, out_ptr, srcs, n), "ucg_builtin_dev_reduce_tree")


def oneshot_reduce_scatter(ctx, peers, out_ptr, count, dt, op, rank, world):
    """out[0:hi-lo] = V(rank, log2 world) over shard [lo, hi) of every member's
    buffer, read in place through `peers` (no staging copy). The caller must
    have all members' inputs complete before, and keep them until all members
    finished (barrier on both sides)."""
    size = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
    lo, hi = shard_bounds(count, size, world, rank)
    srcs = [p + lo * size for p in peers.ptrs]
    _combine_shard(ctx, op, dt, out_ptr, srcs, rank, world, hi - lo)
    return lo, hi


def oneshot_all_gather(ctx, shard_peers, out_ptr, count, dt, world):
    """out = the concatenation of every member's shard (shard_bounds layout),
    read in place from `shard_peers` (PeerBuffers over each member's shard
    buffer) in one launch; the unequal last shard, if any, in a second."""
    size = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
    lo0, hi0 = shard_bounds(count, size, world, 0)
    per = (hi0 - lo0) * size
    lo_l, hi_l = shard_bounds(count, size, world, world - 1)
    last = (hi_l - lo_l) * size
    if world == 1 or last == per:
        _lib.check(ctx.gather_multi(out_ptr, shard_peers.ptrs, per), "gather_multi")
        return
    _lib.check(ctx.gather_multi(out_ptr, shard_peers.ptrs[:-1], per), "gather_multi")
    _lib.check(ctx.gather_multi(out_ptr + lo_l * size, shard_peers.ptrs[-1:], last),
               "gather_multi")


def _gather_rows(ctx, out_ptr, ptrs, rows, count, size, world):
    """out[shard r] = ptrs[r][0 : len(shard r)] for every r in `rows` (member
    indices), in as few launches as the shard_bounds layout allows: one for
    all equal-sized rows - rows not gathered are passed as NULL and left in
    place, so the launch still reads every peer at once - and one for an
    unequal last row."""
    lo0, hi0 = shard_bounds(count, size, world, 0)
    per = (hi0 - lo0) * size
    lo_l, hi_l = shard_bounds(count, size, world, world - 1)
    last = (hi_l - lo_l) * size
    nrows = world if last == per else world - 1
    srcs = [ptrs[r] if r in rows else None for r in range(nrows)]
    if any(p is not None for p in srcs):
        _lib.check(ctx.gather_multi(out_ptr, srcs, per), "ucg_builtin_dev_gather_multi")
    if nrows < world and world - 1 in rows:
        _lib.check(ctx.gather_multi(out_ptr + lo_l * size, [ptrs[world - 1]], last),
                   "ucg_builtin_dev_gather_multi")


def oneshot_allreduce(ctx, send_peers, recv_peers, count, dt, op, rank, world, barrier):
    """Allreduce in two one-shot launches over peer-mapped buffers (xGMI):

      1. reduce-scatter: member r reads shard r of every member's send buffer
         (send_peers) and writes V(r, log2 N) - the reference recursive-doubling
         plan's per-element association (builtin_recursive.c:158-169) - into
         shard r of its own recv buffer;
      2. barrier();
      3. all-gather: member r reads every other shard from its owner's recv
         buffer (recv_peers), all peers at once;
      4. barrier() - no member may overwrite its recv buffer (the next
         operation's step 1) while a peer still reads it.

    Same result as the plan on every member, bit for bit, for a commutative op
    (every member's V(self, log2 N) pairs the same subsets); it moves
    2 (N-1)/N x S per member instead of the plan's log2(N) x S, over all N-1
    links at once instead of one link per step. `barrier` must order the
    device work of all members: a stream-ordered collective (RCCL all_reduce
    of one element on the launch stream) or, for members sharing one GPU in
    tests, ctx.sync() + a host barrier."""
    size = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
    lo, hi = shard_bounds(count, size, world, rank)
    out = recv_peers.ptrs[rank]
    srcs = [p + lo * size for p in send_peers.ptrs]
    _combine_shard(ctx, op, dt, out + lo * size, srcs, rank, world, hi - lo)
    barrier()
    if world > 1:
        shard_ptrs = [p + shard_bounds(count, size, world, r)[0] * size
                      for r, p in enumerate(recv_peers.ptrs)]
        _gather_rows(ctx, out, shard_ptrs, [r for r in range(world) if r != rank], count,
                     size, world)
    barrier()


def oneshot_reduce(ctx, send_peers, out_ptr, count, dt, op, rank, world, root):
    """MPI_Reduce to `root` in one launch (AGGREGATE|SINGLE_DESTINATION,
    which the reference always runs as the tree fan-in, builtin.c:95-121):
    the root reads every member's send buffer in place through `send_peers`
    (all N-1 links at once) and writes the fan-in association of
    builtin_tree.c:262-380 - its own data first, then the children in
    ascending order - into out_ptr. The other members launch nothing; the
    caller's barrier after the call keeps their buffers alive until the root
    is done. Returns True on the root."""
    if rank != root:
        return False
    order = [root] + [m for m in range(world) if m != root]
    _lib.check(ctx.reduce_tree(op, dt, out_ptr, [send_peers.ptrs[m] for m in order], count),
               "ucg_builtin_dev_reduce_tree")
    return True


def stage_slot_bytes(count, elem_size, world):
    """Slot size of the push reduce-scatter's stage: the largest shard (the
    last one), rounded up to 256 B."""
    lo, hi = shard_bounds(count, elem_size, world, world - 1)
    return ((hi - lo) * elem_size + 255) // 256 * 256


def _copy_pairs(ctx, pairs):
    """pairs: (dst, src, nbytes); one copy_multi launch per distinct size."""
    by_size = {}
    for d, s_, n in pairs:
        by_size.setdefault(n, []).append((d, s_))
    for n, ps in by_size.items():
        for i in range(0, len(ps), 16):
            chunk = ps[i:i + 16]
            _lib.check(ctx.copy_multi([d for d, _ in chunk], [s_ for _, s_ in chunk], n),
                       "ucg_builtin_dev_copy_multi")


def push_reduce_scatter(ctx, x_ptr, stage_peers, out_ptr, count, dt, op, rank, world,
                        barrier):
    """The push form of the one-shot reduce-scatter, for links that move
    writes better than reads:

      1. member r writes shard p of its buffer x into slot r of member p's
         stage, all peers at once (one copy_multi launch);
      2. barrier();
      3. member r combines its stage's slots (slot r read in place from x) in
         the plan's association: out = V(r, log2 N) (reduce_multi, self = r).

    stage_peers maps every member's stage of `world` slots of
    stage_slot_bytes(). Same result, bit for bit, as oneshot_reduce_scatter.
    The caller's next barrier must pass before any member writes into the
    stages again. Returns the shard's [lo, hi)."""
    size = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
    slot = stage_slot_bytes(count, size, world)
    pairs = []
    for p in range(world):
        if p != rank:
            plo, phi = shard_bounds(count, size, world, p)
            pairs.append((stage_peers.ptrs[p] + rank * slot, x_ptr + plo * size,
                          (phi - plo) * size))
    _copy_pairs(ctx, pairs)
    barrier()
    lo, hi = shard_bounds(count, size, world, rank)
    stage = stage_peers.ptrs[rank]
    srcs = [x_ptr + lo * size if m == rank else stage + m * slot for m in range(world)]
    _combine_shard(ctx, op, dt, out_ptr, srcs, rank, world, hi - lo)
    return lo, hi


def push_allreduce(ctx, x_ptr, stage_peers, recv_peers, count, dt, op, rank, world,
                   barrier):
    """Allreduce by pushes only: push_reduce_scatter into this member's shard
    of its recv buffer, then the reduced shard written into every peer's recv
    buffer at the same offset (one copy_multi launch), then barrier(). A
    member's pushes land only on the peers' copies of its own shard, which no
    peer writes meanwhile, so one barrier in the middle suffices."""
    size = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
    out = recv_peers.ptrs[rank]
    lo, hi = shard_bounds(count, size, world, rank)
    push_reduce_scatter(ctx, x_ptr, stage_peers, out + lo * size, count, dt, op, rank,
                        world, barrier)
    _copy_pairs(ctx, [(recv_peers.ptrs[p] + lo * size, out + lo * size, (hi - lo) * size)
                      for p in range(world) if p != rank])
    barrier()


def stream_barrier(dist, device, group=None):
    """A barrier on the device streams of all members, without a host sync:
    an RCCL all_reduce of one element enqueued on the current stream completes
    only after every member's earlier work on its stream has (each member's
    contribution is sent after that work), and later work waits for it."""
    import torch
    flag = torch.zeros(1, dtype=torch.int32, device=device)

    def barrier():
        dist.all_reduce(flag, group=group)
    return barrier

"""The reference builtin planner's plans restated in Python, and a
simulation that runs every member's plan to produce the expected results.

TEST INFRASTRUCTURE ONLY (like the rest of oracle/): imported by tests/ as
the checker of the operation engine's plans (xucg_amd/csrc/builtin_plan.c),
never by the product package.

Restated from (paths relative to the reference tree):
  add_intra      builtin/plan/builtin_tree.c:262-380  (root 0)
  add_inter      builtin/plan/builtin_tree.c:382-438
  tree_connect   builtin/plan/builtin_tree.c:86-260   (aggregating modifiers)
  tree plan      builtin/plan/builtin_tree.c:441-561
  recursive plan builtin/plan/builtin_recursive.c:20-228
  topology       builtin/builtin.c:94-131
  buffers        builtin/ops/builtin_control.c:673-683, 755-869, 960-972
with the reference's defects on these paths replaced by their intent (the
list is DESIGN.md 7's table):
  - a host master of a multi-host recursive plan drops its parent from the
    intra-host pass (builtin_recursive.c:55 tests master_phase == HOST, which
    a NET parent never produces);
  - REDUCE_WAYPOINT reduces into the member's accumulator (the reference
    aggregates it as WRITE into an uninitialised temp buffer,
    builtin_control.c:814-819, 960-972);
  - a sending step sends recv.buffer once the member received anything (the
    reference's root sends send.buffer on its host fan-out after a net
    fan-out, builtin_control.c:674-683);
  - a two-level host tree over more than two sockets (or with CACHE
    distances) is Unsupported: the host master takes only the first other
    socket's master as a child (builtin_tree.c:336-351);
  - a root other than 0 is served by the root-0 plan in a numbering where
    the root's host comes first and the root first in it
    (ucg_builtin_topo_tree_set_root, builtin_tree.c:563-608, reads tree
    parameters out of a plan phase).
"""
from . import oracle as O

SELF, CACHE, SOCKET, HOST, NET, LAST = 0, 1, 7, 15, 253, 255   # api/ucg.h:253-264
TREE_MAX_RADIX = 128                                            # builtin_plan.h:98


class Unsupported(Exception):
    pass


def layout(n, my, ppn=None, socket=None):
    """Distance array of member `my` (api/ucg.h:304-322): hosts of `ppn`
    consecutive members, sockets of `socket` consecutive members."""
    ppn = ppn or n
    d = []
    for m in range(n):
        if m == my:
            d.append(SELF)
        elif m // ppn != my // ppn:
            d.append(NET)
        elif socket and m // socket != my // socket:
            d.append(HOST)
        else:
            d.append(SOCKET if socket else HOST)
    return d


def add_intra(d, my, sock_thresh):
    """ucg_builtin_tree_add_intra (root 0): ppn, up, down, master_phase."""
    n = len(d)
    ppn = sum(1 for x in d if x <= HOST)
    single = ppn < sock_thresh

    def dist(m):
        return HOST if (single and d[m] == SOCKET) else d[m]
    up, master_phase, up_distance = [], NET, LAST
    for m in range(my):
        if up_distance > dist(m):
            up_distance = dist(m)
            master_phase = up_distance - 1
            up = [m]
    down, down_distance, first_distance = [], SELF, SELF
    for m in range(my + 1, n):
        x = dist(m)
        if down_distance < x <= master_phase and x < NET:
            down_distance = x
            first_distance = x if first_distance == SELF else LAST
            # the new distance's first member goes to the front, the old
            # front to the back
            down = [m] + down[1:] + down[:1]
        elif x == first_distance:
            down.append(m)
        if len(down) == TREE_MAX_RADIX:
            raise Unsupported("PPN limit")
    return ppn, up, down, master_phase


def check_host_tree(d, sock_thresh):
    """Raise Unsupported for the intra-host trees add_intra cannot build: the
    host master takes the first other socket's master as a child and no later
    one (first_distance turns LAST, builtin_tree.c:336-351), so a host of more
    than two sockets (or a CACHE level inside a socket) leaves masters whose
    parent does not expect them."""
    ppn = sum(1 for x in d if x <= HOST)
    if CACHE in d:
        raise Unsupported("CACHE distances (a third intra-host level)")
    sock = sum(1 for x in d if x <= SOCKET)
    if ppn >= sock_thresh and SOCKET in d and (ppn % sock or ppn // sock > 2):
        raise Unsupported("two-level host tree with more than two sockets")


def add_inter(n, my, ppn, radix):
    """ucg_builtin_tree_add_inter: the masters' tree, root 0."""
    up, down = [], []
    inner_range, outer_range = ppn, ppn * radix
    while True:
        for outer in range(0, n, outer_range):
            root = outer if outer_range < n else 0
            for inner in range(outer, min(outer + outer_range, n), inner_range):
                if my == inner:
                    if my != root:
                        up.append(root)
                elif my == root:
                    down.append(inner)
        inner_range *= radix
        outer_range *= radix
        if not outer_range < n * radix:
            return up, down


def _phase(method, step, peers):
    """Sends and receives of one phase (builtin_control.c:375-396)."""
    p = {"method": method, "step": step, "send": [], "recv": [], "recv_first": False,
         "agg": "nop"}
    if method in ("SEND_TERMINAL", "SEND_TO_SM_ROOT"):
        p["send"] = list(peers)
    elif method == "REDUCE_TERMINAL":
        p["recv"], p["agg"] = list(peers), "reduce"
    elif method == "RECV_TERMINAL":
        p["recv"], p["agg"] = list(peers), "write"
    elif method == "REDUCE_RECURSIVE":
        p["send"], p["recv"], p["agg"] = list(peers), list(peers), "reduce"
    elif method == "REDUCE_WAYPOINT":
        p["recv"], p["send"], p["agg"], p["recv_first"] = list(peers[:-1]), [peers[-1]], \
            "reduce", True
    elif method == "BCAST_WAYPOINT":
        p["recv"], p["send"], p["agg"], p["recv_first"] = [peers[0]], list(peers[1:]), \
            "write", True
    return p


def tree_connect(fanin, fanout, offset, ppn, host_up, net_up, net_down, host_down):
    out = []
    if fanin and host_up + host_down:
        if host_down:
            m = "REDUCE_WAYPOINT" if host_up else "REDUCE_TERMINAL"
        else:
            m = "SEND_TERMINAL" if ppn == 2 else "SEND_TO_SM_ROOT"
        out.append(_phase(m, offset, host_down + host_up[:1]))
    if fanin and net_up + net_down:
        if net_down:
            m = "REDUCE_WAYPOINT" if net_up else "REDUCE_TERMINAL"
        else:
            m = "SEND_TERMINAL"
        out.append(_phase(m, offset + 1, net_down + net_up[:1]))
    if fanout and net_up + net_down:
        if net_down:
            m = "BCAST_WAYPOINT" if net_up else "SEND_TERMINAL"
        else:
            m = "RECV_TERMINAL"
        out.append(_phase(m, offset + 2, net_up + net_down))
    if fanout and host_up + host_down:
        if host_down:
            m = "BCAST_WAYPOINT" if host_up else "SEND_TERMINAL"
        else:
            m = "RECV_TERMINAL"
        out.append(_phase(m, offset + 3, host_up + host_down))
    return out


def tree_plan(d, my, radix, sock_thresh, fanout):
    n = len(d)
    check_host_tree(d, sock_thresh)
    ppn, up, down, mp = add_intra(d, my, sock_thresh)
    net_up, net_down = [], []
    if mp >= HOST and ppn < n:
        up = []
        net_up, net_down = add_inter(n, my, ppn, radix)
    return "tree", ppn, tree_connect(True, fanout, 1, ppn, up, net_up, net_down, down)


def recursive_plan(d, my, factor, sock_thresh):
    n = len(d)
    ppn, up, down, mp = add_intra(d, my, sock_thresh)
    if mp >= HOST:
        up = []
    if factor < 2:
        raise Unsupported("factor < 2")
    procs = ppn if n == ppn else n // ppn + (n % ppn > 0)
    steps, size = 0, 1
    while size < procs:
        size *= factor
        steps += 1
    if size != procs:
        if n != ppn:
            raise Unsupported("hosts not a power of the factor")
        steps = 0
    plan_ppn = ppn
    if n == ppn and steps:
        up, down, ppn = [], [], 1
    else:
        check_host_tree(d, sock_thresh)
    phases = []
    if up or down:
        phases += tree_connect(True, False, 1, ppn, up, [], [], down)
    if not up:
        idx = len(phases) + 1
        size = ppn
        for k in range(steps):
            base = my - my % (size * factor)
            peers = [base + (my - base + size * j) % (size * factor) for j in range(1, factor)]
            phases.append(_phase("REDUCE_RECURSIVE", idx + k, peers))
            size *= factor
    if up or down:
        phases += tree_connect(False, True, steps + 1, ppn, up, [], [], down)
    name = "tree" if steps == 0 else "recursive"
    return name, plan_ppn, phases


def virtual_order(n, ppn, root):
    """v2r: the root's host first, the root first in it."""
    H, hr, lr = n // ppn, root // ppn, root % ppn
    v2r = []
    for v in range(n):
        vb, vi = divmod(v, ppn)
        li = vi if vb else (lr if vi == 0 else (vi - 1 if vi <= lr else vi))
        v2r.append(((vb + hr) % H) * ppn + li)
    return v2r


def plan(kind, n, my, ppn=None, socket=None, root=0, radix=8, sock_thresh=16, factor=2,
         force=None):
    """Member `my`'s phases for kind "allreduce" or "reduce" (real member
    indices). force: None, "tree" or "recursive" (UCX_BUILTIN_ALLREDUCE_PLAN)."""
    ppn = ppn or n
    if n % ppn:
        raise Unsupported("hosts of different sizes")
    v2r = virtual_order(n, ppn, root)
    r2v = {r: v for v, r in enumerate(v2r)}
    d_real = layout(n, my, ppn, socket)
    d = [d_real[v2r[v]] for v in range(n)]
    if root != 0:
        d = [HOST if x == SOCKET else x for x in d]
    vmy = r2v[my]
    if n == 1:
        return "none", 1, []
    if kind == "reduce":
        name, pp, phases = tree_plan(d, vmy, radix, sock_thresh, False)
    else:
        use_tree = (n & (n - 1)) != 0 if force is None else force == "tree"
        name, pp, phases = (tree_plan(d, vmy, radix, sock_thresh, True) if use_tree else
                            recursive_plan(d, vmy, factor, sock_thresh))
    for p in phases:
        p["send"] = [v2r[x] for x in p["send"]]
        p["recv"] = [v2r[x] for x in p["recv"]]
    return name, pp, phases


def simulate(kind, op, dt, inputs, root=0, **cfg):
    """Run every member's plan with whole-buffer messages; children's data is
    applied in each step's peer order (the engine applies arrival order: the
    results agree whenever the association does not matter - integers, exact
    floats). Returns the members' recv buffers (reduce: the root's only,
    others None). Raises RuntimeError if the plans do not fit together (a
    message nobody expects, or a member waiting forever)."""
    n = len(inputs)
    plans = [plan(kind, n, m, root=root, **cfg)[2] for m in range(n)]
    acc = [x.copy() for x in inputs]     # init_reduce where it matters
    got_any = [False] * n
    cur = [0] * n
    sent = [False] * n                   # sends of the current phase done
    box = {}                             # (dst, step, src) -> data

    def send(m, p):
        buf = acc[m] if (got_any[m] or p["recv_first"]) else inputs[m]
        for q in p["send"]:
            key = (q, p["step"], m)
            if key in box:
                raise RuntimeError(f"duplicate message {key}")
            box[key] = buf.copy()

    progress = True
    while progress:
        progress = False
        for m in range(n):
            while cur[m] < len(plans[m]):
                p = plans[m][cur[m]]
                if not p["recv_first"] and not sent[m]:
                    send(m, p)
                    sent[m] = True
                    progress = True
                if not all((m, p["step"], s) in box for s in p["recv"]):
                    break
                for s in p["recv"]:
                    data = box.pop((m, p["step"], s))
                    acc[m] = O.reduce(op, dt, data, acc[m]) if p["agg"] == "reduce" else data
                if p["recv"]:
                    got_any[m] = True
                if p["recv_first"]:
                    send(m, p)
                cur[m] += 1
                sent[m] = False
                progress = True
    if any(cur[m] < len(plans[m]) for m in range(n)) or box:
        raise RuntimeError(f"plans do not fit: positions {cur}, undelivered {sorted(box)}")
    if kind == "reduce":
        return [acc[m] if m == root else None for m in range(n)]
    return acc

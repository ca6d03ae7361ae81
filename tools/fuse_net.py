"""Three-input fusion of the k-select merge networks (csrc/sra_common.hpp).

The trimmed-mean network of select_plain_kernel<1, 128, 12> is 32 sorted
4-blocks followed by Batcher odd-even merges pruned to the kept ranks
[12, 116).  Inside a merge every intermediate value is read by exactly one
later compare-exchange, and a value v = min(p, q) read only by a CE (v, w)
can be dropped:

    min(v, w) = min3(p, q, w)                       always,
    max(v, w) = med3(p, q, w)    iff w <= max(p, q) for every input,

(symmetrically v = max(p, q): max(v, w) = max3(p, q, w), min(v, w) =
med3(p, q, w) iff w >= min(p, q)).  min3 / med3 / max3 are single VALU ops
on gfx950 that read three registers, the pair they replace read four, so
each fusion removes one instruction and no register read.

Validity is checked with the 0-1 principle: every op here commutes with
monotone maps, so a condition that holds for every 0-1 input of a merge
(two sorted 0-1 halves: (n/2 + 1)^2 inputs) holds for every real input.
The fused program of the whole network is then checked against np.sort on
random real columns with ties.

usage: python tools/fuse_net.py --emit-all secure-robust-federated-learning_amd/csrc/net_fused.inc
       python tools/fuse_net.py [--p2 --pr --olo --ohi]   (count and check one network)
"""
from __future__ import annotations

import argparse
import itertools
import sys

import numpy as np

CE, MIN, MAX, MOVE = 0, 1, 2, 3
MIN3, MAX3, MED3 = 4, 5, 6


# ---------------------------------------------------------------------------
# the planner of sra_common.hpp (BaseNet / NetPlanData), restated
# ---------------------------------------------------------------------------
def merge_stages(out, lo, n, tag):
    p = n // 2
    k = p
    while k >= 1:
        j = k % p
        while j + k < n:
            i = 0
            while i < k and i + j + k < n:
                out.append((lo + i + j, lo + i + j + k, tag))
                i += 1
            j += 2 * k
        k //= 2


def merge_rec(out, lo, n, r, tag):
    """Batcher's odd-even merge in recursive (depth-first) order: the same
    comparators as merge_stages, but a comparator's consumer follows it
    closely, which keeps the fused program's live values near 128 (137 slots
    at N = 128 against 169 in stage-major order)."""
    step = r * 2
    if step < n:
        merge_rec(out, lo, n, step, tag)
        merge_rec(out, lo + r, n, step, tag)
        i = lo + r
        while i + r < lo + n:
            out.append((i, i + r, tag))
            i += step
    else:
        out.append((lo, lo + r, tag))


def from4(out, lo, n, tags):
    if n <= 4:
        return
    from4(out, lo, n // 2, tags)
    from4(out, lo + n // 2, n // 2, tags)
    tags.append((lo, n, "merge"))
    merge_rec(out, lo, n, 1, len(tags) - 1)


def bitonic_rec(out, lo, n, tag):
    """Half-cleaner cascade (network_plain<..., kNetMerge>: sorts a bitonic
    sequence) in depth-first order: the half-clean of [lo, lo + n), then each
    half."""
    if n < 2:
        return
    h = n // 2
    for i in range(h):
        out.append((lo + i, lo + i + h, tag))
    bitonic_rec(out, lo, h, tag)
    bitonic_rec(out, lo + h, h, tag)


def plan(p2, pr, olo, ohi, net="from4"):
    """Forward fold of the compile-time top pads, backward cone pruning: the
    op list network_plain<P2, PR, OLO, OHI, kNetFrom4 / kNetMerge> runs
    (kind, a, b, unit)."""
    base, tags = [], []
    if net == "from4":
        from4(base, 0, p2, tags)
    else:
        tags.append((0, p2, "bitonic"))
        bitonic_rec(base, 0, p2, 0)
    cst = [i >= pr for i in range(p2)]
    ops = []
    for x, y, t in base:
        if cst[y]:
            continue
        if cst[x]:
            ops.append([MOVE, x, y, t])
            cst[x], cst[y] = False, True
            continue
        ops.append([CE, x, y, t])
    need = [olo <= i < ohi for i in range(p2)]
    keep = [False] * len(ops)
    for q in range(len(ops) - 1, -1, -1):
        k, x, y, t = ops[q]
        if k == MOVE:
            keep[q] = need[x]
            need[y] = need[x]
            need[x] = False
            continue
        nx, ny = need[x], need[y]
        if not nx and not ny:
            continue
        keep[q] = True
        ops[q][0] = CE if (nx and ny) else (MIN if nx else MAX)
        need[x] = need[y] = True
    return [tuple(o) for o, kp in zip(ops, keep) if kp], tags


# ---------------------------------------------------------------------------
# SSA form
# ---------------------------------------------------------------------------
class Val:
    __slots__ = ("id", "kind", "args", "consumers", "dead")

    def __init__(self, vid, kind, args):
        self.id, self.kind, self.args, self.consumers, self.dead = vid, kind, list(args), [], False


def to_ssa(ops, p2):
    """values[i]: kind in {None (input), MIN, MAX, MIN3, MAX3, MED3}; returns
    (values, slot_final, op_outputs) with op_outputs[q] = (lo value, hi value)."""
    vals = [Val(i, None, ()) for i in range(p2)]
    slot = list(range(p2))
    op_out = []
    for k, x, y, t in ops:
        if k == MOVE:
            slot[x] = slot[y]
            op_out.append((None, None))
            continue
        a, b = slot[x], slot[y]
        lo = hi = None
        if k in (CE, MIN):
            lo = len(vals)
            vals.append(Val(lo, MIN, (a, b)))
            slot[x] = lo
        if k in (CE, MAX):
            hi = len(vals)
            vals.append(Val(hi, MAX, (a, b)))
            slot[y] = hi
        for u in (a, b):
            for o in (lo, hi):
                if o is not None:
                    vals[u].consumers.append(o)
        op_out.append((lo, hi))
    return vals, slot


def merge_of_value(vals, v, op_merge):
    return op_merge.get(v)


def zero_one_inputs(n, kind="merge"):
    """All 0-1 inputs of a unit: a merge of two sorted halves of n/2 values,
    or a bitonic sequence of n (0^a 1^b 0^c and 1^a 0^b 1^c)."""
    rows = []
    if kind == "merge":
        h = n // 2
        for z1 in range(h + 1):
            for z2 in range(h + 1):
                rows.append([0] * z1 + [1] * (h - z1) + [0] * z2 + [1] * (h - z2))
    else:
        for a in range(n + 1):
            for b in range(n + 1 - a):
                c = n - a - b
                rows.append([0] * a + [1] * b + [0] * c)
                rows.append([1] * a + [0] * b + [1] * c)
    return np.array(rows, dtype=np.int8)


def fuse(ops, tags, p2, olo, ohi, verbose=False):
    vals, final_slot = to_ssa(ops, p2)
    # merge membership of each produced value (the op's merge tag)
    op_merge = {}
    vi = p2
    for k, x, y, t in ops:
        if k == MOVE:
            continue
        if k in (CE, MIN):
            op_merge[vi] = t
            vi += 1
        if k in (CE, MAX):
            op_merge[vi] = t
            vi += 1
    # evaluate every value on every 0-1 input of its merge (inputs of the merge
    # = the slot values when the merge starts)
    tag_inputs = {}
    slot = list(range(p2))
    ev = {}          # value id -> (tag, int8 vector over that merge's 0-1 inputs)
    cur_tag = None
    vi = p2
    for k, x, y, t in ops:
        if t != cur_tag:
            cur_tag = t
            lo, n, kind = tags[t]
            Z = zero_one_inputs(n, kind)
            for s in range(lo, lo + n):
                ev[slot[s]] = (t, Z[:, s - lo])
        if k == MOVE:
            slot[x] = slot[y]
            continue
        a, b = slot[x], slot[y]
        va, vb = ev[a][1], ev[b][1]
        if k in (CE, MIN):
            ev[vi] = (t, np.minimum(va, vb))
            slot[x] = vi
            vi += 1
        if k in (CE, MAX):
            ev[vi] = (t, np.maximum(va, vb))
            slot[y] = vi
            vi += 1
    outputs = set(final_slot[olo:ohi])
    fused = 0
    for v in vals:
        if v.kind not in (MIN, MAX) or v.dead or v.id in outputs:
            continue
        if len(set(v.consumers)) == 0:
            continue
        cons = sorted(set(v.consumers))
        # v's consumers: the one or two outputs of ONE later op (same args)
        args0 = tuple(vals[cons[0]].args)
        if any(tuple(vals[c].args) != args0 for c in cons) or len(cons) > 2:
            continue
        if any(vals[c].kind not in (MIN, MAX) for c in cons):
            continue
        if any(vals[a].kind is not None and vals[a].dead for a in v.args):
            continue
        p, q = v.args
        if vals[p].dead or vals[q].dead:
            continue
        w = args0[0] if args0[1] == v.id else args0[1]
        if w == v.id:
            continue
        t = op_merge[v.id]
        # every value involved must belong to the same merge's evaluation
        if any(x not in ev or ev[x][0] != t for x in (p, q, w)) or any(op_merge.get(c) != t for c in cons):
            continue
        ep, eq, ew = ev[p][1], ev[q][1], ev[w][1]
        ok = True
        new = {}
        for c in cons:
            ck = vals[c].kind
            if v.kind == MIN and ck == MIN:
                new[c] = MIN3
            elif v.kind == MAX and ck == MAX:
                new[c] = MAX3
            elif v.kind == MIN and ck == MAX:          # max(w, min(p,q)) = med3 iff w <= max(p,q)
                ok &= bool(np.all(ew <= np.maximum(ep, eq)))
                new[c] = MED3
            else:                                       # min(w, max(p,q)) = med3 iff w >= min(p,q)
                ok &= bool(np.all(ew >= np.minimum(ep, eq)))
                new[c] = MED3
        if not ok:
            continue
        for c, nk in new.items():
            vals[c].kind = nk
            vals[c].args = [p, q, w]
        v.dead = True
        # p, q, w gain the consumers; v disappears
        for c in cons:
            vals[p].consumers.append(c)
            vals[q].consumers.append(c)
        fused += 1
    return vals, final_slot, fused


def count_ops(vals, p2):
    return sum(1 for v in vals[p2:] if not v.dead)


def evaluate(vals, p2, X):
    """Run the (fused) SSA program on the columns of X (p2 x m)."""
    r = [None] * len(vals)
    for i in range(p2):
        r[i] = X[i]
    for v in vals[p2:]:
        if v.dead:
            continue
        a = [r[u] for u in v.args]
        if v.kind == MIN:
            r[v.id] = np.minimum(a[0], a[1])
        elif v.kind == MAX:
            r[v.id] = np.maximum(a[0], a[1])
        elif v.kind == MIN3:
            r[v.id] = np.minimum(np.minimum(a[0], a[1]), a[2])
        elif v.kind == MAX3:
            r[v.id] = np.maximum(np.maximum(a[0], a[1]), a[2])
        else:
            r[v.id] = np.maximum(np.minimum(a[0], a[1]), np.minimum(np.maximum(a[0], a[1]), a[2]))
    return r


def random_inputs(p2, pr, net, trials, seed):
    """Random columns with many ties in the network's input form (sorted
    4-blocks of pr values + top pads, or a bitonic sequence) and their sort."""
    rng = np.random.default_rng(seed)
    X = rng.integers(-40, 40, size=(pr, trials)).astype(np.float64)
    X[:, : trials // 2] = rng.standard_normal((pr, trials // 2))
    want = np.sort(X, axis=0)
    if net == "from4":
        for b in range(0, pr, 4):
            X[b:b + 4] = np.sort(X[b:b + 4], axis=0)
    else:
        cut = rng.integers(0, pr + 1, trials)
        for j in range(trials):        # ascending to a peak, then descending (or the mirror)
            k = cut[j]
            col = np.concatenate([np.sort(X[:k, j]), np.sort(X[k:, j])[::-1]])
            X[:, j] = col if j % 2 else col[::-1]
    full = np.vstack([X, np.full((p2 - pr, trials), np.inf)])
    return full, want


def check(vals, final_slot, p2, pr, olo, ohi, trials=20000, seed=0, net="from4"):
    full, want = random_inputs(p2, pr, net, trials, seed)
    r = evaluate(vals, p2, full)
    for s in range(olo, ohi):
        if not np.array_equal(r[final_slot[s]], want[s]):
            return False
    return True


KIND_NAME = {MIN: "min", MAX: "max", MIN3: "min3", MAX3: "max3", MED3: "med3"}


def interleave(live, group=4, window=24):
    """Order the program for its inline-asm form (``group`` ops per asm
    statement): the compiler puts an s_nop before an asm statement that reads
    a register the asm statement just before it wrote (the gfx950 dst-forwarding
    hazard rule applied to asm it cannot look into).  Greedy list order: fill
    each group with the earliest ready ops (within ``window`` of the earliest
    ready one, which bounds the live set) that read nothing the previous group
    produced; reads of the current group's own results are fine."""
    first = min(v.id for v in live) if live else 0
    done = set(range(first))
    produced = {v.id for v in live}
    pending = list(live)
    out = []
    prev_group, cur_group = set(), set()
    while pending:
        ready = [q for q, v in enumerate(pending[:window * 4])
                 if all(a in done or a not in produced or a in cur_group for a in v.args)]
        pick = ready[0]
        for q in ready:
            if q - ready[0] > window:
                break
            if not any(a in prev_group for a in pending[q].args):
                pick = q
                break
        v = pending.pop(pick)
        out.append(v)
        cur_group.add(v.id)
        if len(cur_group) == group:
            done |= cur_group
            prev_group, cur_group = cur_group, set()
    return out


def allocate(vals, final_slot, p2, olo, ohi):
    """Slot allocation of the fused SSA program (register-array slots with
    compile-time indices in the kernel): a slot is reused once its value's
    last reader has run; the op writes in place of a dying argument where it
    can.  Returns (ops [(kind, dst, a, b, c)], out_slots, nslots)."""
    live = interleave([v for v in vals[p2:] if not v.dead], GROUP)
    pos = {v.id: q for q, v in enumerate(live)}
    outputs = [final_slot[s] for s in range(olo, ohi)]
    last = {}
    for q, v in enumerate(live):
        for u in v.args:
            last[u] = q
    for u in outputs:
        last[u] = len(live)
    slot_of = {i: i for i in range(p2)}
    free = sorted(i for i in range(p2) if i not in last)
    nslots = p2
    prog = []
    for q, v in enumerate(live):
        args = [slot_of[u] for u in v.args]
        dying = [slot_of[u] for u in dict.fromkeys(v.args) if last.get(u) == q]
        if dying:
            dst = dying[0]
            free.extend(dying[1:])
        elif free:
            dst = free.pop(0)
        else:
            dst = nslots
            nslots += 1
        free.sort()
        slot_of[v.id] = dst
        prog.append((v.kind, dst, args[0], args[1], args[2] if len(args) > 2 else args[1]))
    return prog, [slot_of[u] for u in outputs], nslots


def emit(path, name, prog, outs, nslots, info):
    k = {MIN: 1, MAX: 2, MIN3: 3, MAX3: 4, MED3: 5}
    with open(path, "w") as f:
        f.write("// Generated by tools/fuse_net.py -- do not edit.\n")
        f.write("// %s\n" % info)
        f.write("// ops: 1 min, 2 max, 3 min3, 4 max3, 5 med3 (dst, a, b, c); slot indices into v[kSlots].\n")
        f.write("struct %s {\n" % name)
        f.write("  static constexpr int kSlots = %d;\n" % nslots)
        f.write("  static constexpr int kOps = %d;\n" % len(prog))
        f.write("  static constexpr int kOuts = %d;\n" % len(outs))
        for nm, col in (("kKind", [k[p[0]] for p in prog]), ("kDst", [p[1] for p in prog]),
                        ("kA", [p[2] for p in prog]), ("kB", [p[3] for p in prog]), ("kC", [p[4] for p in prog])):
            f.write("  static constexpr short %s[%d] = {" % (nm, len(col)))
            for i, x in enumerate(col):
                if i % 24 == 0:
                    f.write("\n      ")
                f.write("%d," % x)
            f.write("};\n")
        f.write("  static constexpr short kOut[%d] = {" % len(outs))
        for i, x in enumerate(outs):
            if i % 24 == 0:
                f.write("\n      ")
            f.write("%d," % x)
        f.write("};\n")
        f.write("  // the program as inline asm, %d ops per statement (one boundary, and at\n" % GROUP)
        f.write("  // most one hazard s_nop, per group instead of per op)\n")
        f.write("  template <int S>\n")
        f.write("  static __device__ __forceinline__ void run(float (&v)[S]) {\n")
        f.write("    static_assert(S >= kSlots, \"register array smaller than the program's slots\");\n")
        for g0 in range(0, len(prog), GROUP):
            f.write(asm_group(prog[g0:g0 + GROUP]))
        f.write("  }\n};\n")


GROUP = 4
ASM = {MIN: "v_min_f32", MAX: "v_max_f32", MIN3: "v_min3_f32", MAX3: "v_max3_f32", MED3: "v_med3_f32"}


def asm_group(ops):
    """One asm statement for consecutive ops: reads of slots not yet written
    in the group are inputs, every op's result an early-clobber output (an
    output must not share a register with an input a later op of the group
    still reads); afterwards each written slot takes its last output."""
    cur = {}            # slot -> ("o", k) once written in the group
    ins, outs_w, lines = [], [], []
    for kind, d, a, b, c in ops:
        args = [a, b] if kind in (MIN, MAX) else [a, b, c]
        refs = []
        for x in args:
            if x in cur:
                refs.append(("o", cur[x]))
            else:
                if x not in ins:
                    ins.append(x)
                refs.append(("i", ins.index(x)))
        k = len(outs_w)
        outs_w.append(d)
        cur[d] = k
        lines.append((ASM[kind], k, refs))
    no = len(outs_w)
    text = "\\n\\t".join("%s %%%d, %s" % (op, k, ", ".join("%%%d" % (r[1] if r[0] == "o" else no + r[1])
                                                                for r in refs)) for op, k, refs in lines)
    decl = ", ".join("o%d" % k for k in range(no))
    cons_o = ", ".join('"=&v"(o%d)' % k for k in range(no))
    cons_i = ", ".join('"v"(v[%d])' % x for x in ins)
    last = {}
    for k, d in enumerate(outs_w):
        last[d] = k
    assign = " ".join("v[%d] = o%d;" % (d, k) for d, k in sorted(last.items()))
    return ("    {\n      float %s;\n      asm(\"%s\"\n          : %s\n          : %s);\n      %s\n    }\n"
            % (decl, text, cons_o, cons_i, assign))


def check_prog(prog, outs, nslots, p2, pr, olo, trials=20000, seed=1, net="from4"):
    """Run the slot-allocated program (what the kernel executes) on random
    inputs and compare the kept ranks with np.sort."""
    X, want = random_inputs(p2, pr, net, trials, seed)
    v = [None] * nslots
    for i in range(p2):
        v[i] = X[i]
    for kind, d, a, b, c in prog:
        if kind == MIN:
            r = np.minimum(v[a], v[b])
        elif kind == MAX:
            r = np.maximum(v[a], v[b])
        elif kind == MIN3:
            r = np.minimum(np.minimum(v[a], v[b]), v[c])
        elif kind == MAX3:
            r = np.maximum(np.maximum(v[a], v[b]), v[c])
        else:
            r = np.maximum(np.minimum(v[a], v[b]), np.minimum(np.maximum(v[a], v[b]), v[c]))
        v[d] = r
    return all(np.array_equal(v[o], want[olo + i]) for i, o in enumerate(outs))


# the programs the k-select kernels run (csrc/net_fused.inc): name, P2, PR,
# kept ranks [OLO, OHI)
PROGRAMS = [
    ("FusedTm128", 128, 128, 12, 116, "from4"),     # trimmed mean N = 128 (the north star)
    ("FusedTm100", 128, 100, 10, 90, "from4"),      # trimmed mean N = 100
    ("FusedMed128", 128, 128, 63, 65, "from4"),     # median N = 128
    ("FusedMed100", 128, 100, 49, 51, "from4"),     # median N = 100
    ("FusedSort128", 128, 128, 0, 128, "from4"),    # select_quad_kernel: each lane's 128 values
    ("FusedBitonic128", 128, 128, 0, 128, "bitonic"),   # select_quad_kernel: in-lane half-cleaners
]


def build(p2, pr, olo, ohi, net="from4"):
    ops, tags = plan(p2, pr, olo, ohi, net)
    n_ops = sum(2 if k == CE else (0 if k == MOVE else 1) for k, *_ in ops)
    vals, final_slot, fused = fuse(ops, tags, p2, olo, ohi)
    if not check(vals, final_slot, p2, pr, olo, ohi, net=net):
        raise SystemExit("fused SSA program fails the np.sort check")
    prog, outs, nslots = allocate(vals, final_slot, p2, olo, ohi)
    if not check_prog(prog, outs, nslots, p2, pr, olo, net=net):
        raise SystemExit("slot program fails the np.sort check")
    info = ("network_plain<%d, %d, %d, %d, %s> after %d three-input fusions: %d -> %d ops, %d slots"
            % (p2, pr, olo, ohi, "kNetFrom4" if net == "from4" else "kNetMerge", fused, n_ops, len(prog), nslots))
    return prog, outs, nslots, info


def emit_all(path):
    with open(path, "w") as f:
        f.write("// Generated by tools/fuse_net.py --emit-all -- do not edit.\n")
        f.write("// Straight-line min / max / min3 / max3 / med3 programs of the k-select\n")
        f.write("// networks (sorted 4-blocks in v[0 .. PR), kept ranks in v[kOut[...]]).\n")
        f.write("// ops: 1 min, 2 max, 3 min3, 4 max3, 5 med3 of slots (a, b, c) into slot dst.\n")
    for name, p2, pr, olo, ohi, net in PROGRAMS:
        prog, outs, nslots, info = build(p2, pr, olo, ohi, net)
        print(name, info)
        tmp = path + ".part"
        emit(tmp, name, prog, outs, nslots, info)
        with open(tmp) as g, open(path, "a") as f:
            f.write("\n" + "".join(g.readlines()[1:]))
        import os
        os.remove(tmp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p2", type=int, default=128)
    ap.add_argument("--pr", type=int, default=128)
    ap.add_argument("--olo", type=int, default=12)
    ap.add_argument("--ohi", type=int, default=116)
    ap.add_argument("--net", default="from4", choices=["from4", "bitonic"])
    ap.add_argument("--emit", default=None)
    ap.add_argument("--name", default="FusedTm128")
    ap.add_argument("--emit-all", default=None, help="write every PROGRAMS entry into one header")
    a = ap.parse_args()
    if a.emit_all:
        emit_all(a.emit_all)
        return
    prog, outs, nslots, info = build(a.p2, a.pr, a.olo, a.ohi, a.net)
    print(info + ", checked against np.sort")
    if a.emit:
        emit(a.emit, a.name, prog, outs, nslots, info)

if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Map the Boyar-Peralta AES S-box circuit (eprint 2009/191: 32 AND + 81 XOR/XNOR) onto 3-input lookup gates --
gfx950's v_bitop3_b32 computes any boolean function of three 32-bit operands in one VALU instruction -- and emit
the mapped circuit as C (tools/bs_probe/bs8_sbox.h).

Cut-based technology mapping: every node's 3-feasible cuts are enumerated, a cover is chosen by area flow and
then improved by exact-area recovery passes with randomised tie-breaks; the best cover found is emitted.  Every
emitted gate's 8-entry truth table is computed from the circuit itself, and the whole mapped S-box is checked here
against the AES S-box on all 256 inputs before anything is written.

    python3 tools/bs_probe/lut3_map.py [--iters N] [--out PATH]
"""
import argparse
import itertools
import os
import random
import sys

# Boyar-Peralta, inputs u0 (MSB) .. u7 (LSB), outputs s0 (MSB) .. s7 (LSB); "^~" = XNOR
CIRCUIT = """
y14 = u3 ^ u5
y13 = u0 ^ u6
y9 = u0 ^ u3
y8 = u0 ^ u5
t0 = u1 ^ u2
y1 = t0 ^ u7
y4 = y1 ^ u3
y12 = y13 ^ y14
y2 = y1 ^ u0
y5 = y1 ^ u6
y3 = y5 ^ y8
t1 = u4 ^ y12
y15 = t1 ^ u5
y20 = t1 ^ u1
y6 = y15 ^ u7
y10 = y15 ^ t0
y11 = y20 ^ y9
y7 = u7 ^ y11
y17 = y10 ^ y11
y19 = y10 ^ y8
y16 = t0 ^ y11
y21 = y13 ^ y16
y18 = u0 ^ y16
t2 = y12 & y15
t3 = y3 & y6
t4 = t3 ^ t2
t5 = y4 & u7
t6 = t5 ^ t2
t7 = y13 & y16
t8 = y5 & y1
t9 = t8 ^ t7
t10 = y2 & y7
t11 = t10 ^ t7
t12 = y9 & y11
t13 = y14 & y17
t14 = t13 ^ t12
t15 = y8 & y10
t16 = t15 ^ t12
t17 = t4 ^ t14
t18 = t6 ^ t16
t19 = t9 ^ t14
t20 = t11 ^ t16
t21 = t17 ^ y20
t22 = t18 ^ y19
t23 = t19 ^ y21
t24 = t20 ^ y18
t25 = t21 ^ t22
t26 = t21 & t23
t27 = t24 ^ t26
t28 = t25 & t27
t29 = t28 ^ t22
t30 = t23 ^ t24
t31 = t22 ^ t26
t32 = t31 & t30
t33 = t32 ^ t24
t34 = t23 ^ t33
t35 = t27 ^ t33
t36 = t24 & t35
t37 = t36 ^ t34
t38 = t27 ^ t36
t39 = t29 & t38
t40 = t25 ^ t39
t41 = t40 ^ t37
t42 = t29 ^ t33
t43 = t29 ^ t40
t44 = t33 ^ t37
t45 = t42 ^ t41
z0 = t44 & y15
z1 = t37 & y6
z2 = t33 & u7
z3 = t43 & y16
z4 = t40 & y1
z5 = t29 & y7
z6 = t42 & y11
z7 = t45 & y17
z8 = t41 & y10
z9 = t44 & y12
z10 = t37 & y3
z11 = t33 & y4
z12 = t43 & y13
z13 = t40 & y5
z14 = t29 & y2
z15 = t42 & y9
z16 = t45 & y14
z17 = t41 & y8
t46 = z15 ^ z16
t47 = z10 ^ z11
t48 = z5 ^ z13
t49 = z9 ^ z10
t50 = z2 ^ z12
t51 = z2 ^ z5
t52 = z7 ^ z8
t53 = z0 ^ z3
t54 = z6 ^ z7
t55 = z16 ^ z17
t56 = z12 ^ t48
t57 = t50 ^ t53
t58 = z4 ^ t46
t59 = z3 ^ t54
t60 = t46 ^ t57
t61 = z14 ^ t57
t62 = t52 ^ t58
t63 = t49 ^ t58
t64 = z4 ^ t59
t65 = t61 ^ t62
t66 = z1 ^ t63
s0 = t59 ^ t63
s6 = t56 ^~ t62
s7 = t48 ^~ t60
t67 = t64 ^ t65
s3 = t53 ^ t66
s4 = t51 ^ t66
s5 = t47 ^ t65
s1 = t64 ^~ s3
s2 = t55 ^~ t67
"""
INPUTS = [f"u{i}" for i in range(8)]
OUTPUTS = [f"s{i}" for i in range(8)]


def parse():
    nodes = {}
    order = []
    for line in CIRCUIT.strip().splitlines():
        dst, expr = [x.strip() for x in line.split("=")]
        if "^~" in expr:
            a, b = [x.strip() for x in expr.split("^~")]
            op = "xnor"
        elif "^" in expr:
            a, b = [x.strip() for x in expr.split("^")]
            op = "xor"
        else:
            a, b = [x.strip() for x in expr.split("&")]
            op = "and"
        nodes[dst] = (op, a, b)
        order.append(dst)
    return nodes, order


def aes_sbox():
    def gmul(a, b):
        p = 0
        while b:
            if b & 1:
                p ^= a
            a = ((a << 1) ^ (0x1b if a & 0x80 else 0)) & 0xff
            b >>= 1
        return p
    S = []
    for x in range(256):
        inv = 0 if x == 0 else next(y for y in range(1, 256) if gmul(x, y) == 1)
        s, r = inv, inv
        for _ in range(4):
            r = ((r << 1) | (r >> 7)) & 0xff
            s ^= r
        S.append(s ^ 0x63)
    return S


OPS = {"xor": lambda a, b: a ^ b, "and": lambda a, b: a & b, "xnor": lambda a, b: 1 - (a ^ b)}


def eval_cone(nodes, root, leaves, vals):
    """value of `root` with the leaves set to vals (dict), recursing through the circuit"""
    memo = dict(zip(leaves, vals))

    def ev(n):
        if n in memo:
            return memo[n]
        op, a, b = nodes[n]
        v = OPS[op](ev(a), ev(b))
        memo[n] = v
        return v
    return ev(root)


def enumerate_cuts(nodes, order, K=3):
    cuts = {u: [frozenset([u])] for u in INPUTS}
    for n in order:
        _, a, b = nodes[n]
        cs = set()
        for ca in cuts[a]:
            for cb in cuts[b]:
                u = ca | cb
                if len(u) <= K:
                    cs.add(u)
        # drop dominated cuts (a superset of another cut of the same node)
        cs = [c for c in cs if not any(d < c for d in cs)]
        cuts[n] = [frozenset([n])] + sorted(cs, key=lambda c: (len(c), sorted(c)))
    return cuts


def cover_size(nodes, choice):
    """LUTs needed when each node n uses cut choice[n]: the nodes reachable from the outputs through chosen cuts"""
    need = set()
    stack = list(OUTPUTS)
    while stack:
        n = stack.pop()
        if n in need or n in INPUTS:
            continue
        need.add(n)
        stack.extend(choice[n])
    return need


def map_circuit(nodes, order, cuts, rng, passes=6):
    fanout = {n: 0 for n in list(nodes) + INPUTS}
    for n in order:
        _, a, b = nodes[n]
        fanout[a] += 1
        fanout[b] += 1
    # area flow with random tie-breaks
    af = {u: 0.0 for u in INPUTS}
    choice = {}
    for n in order:
        best = None
        for c in cuts[n][1:]:
            v = 1.0 + sum(af[l] / max(1, fanout[l]) for l in c) + rng.random() * 1e-3
            if best is None or v < best[0]:
                best = (v, c)
        af[n] = best[0]
        choice[n] = best[1]
    # exact-area recovery: re-choose each needed node's cut to minimise the cover size
    for _ in range(passes):
        improved = False
        need = cover_size(nodes, choice)
        for n in rng.sample(sorted(need), len(need)):
            cur = len(cover_size(nodes, choice))
            best_c, best_v = choice[n], cur
            for c in cuts[n][1:]:
                if c == choice[n]:
                    continue
                old = choice[n]
                choice[n] = c
                v = len(cover_size(nodes, choice))
                choice[n] = old
                if v < best_v or (v == best_v and rng.random() < 0.3):
                    best_c, best_v = c, v
            if best_c != choice[n]:
                improved |= best_v < cur
                choice[n] = best_c
        if not improved:
            break
    return choice, cover_size(nodes, choice)


def topo_emit(nodes, order, choice, need):
    """gates in topological order: (name, [a, b, c], truth table); cuts of fewer than 3 leaves repeat their last
    leaf (the hardware then sees equal bits in those positions, so the other table entries are don't-cares)"""
    pos = {n: i for i, n in enumerate(order)}
    gates = []
    for n in sorted(need, key=lambda x: pos[x]):
        leaves = sorted(choice[n], key=lambda x: (x not in INPUTS, pos.get(x, -1), x))
        leaves = (leaves + [leaves[-1]] * 3)[:3]
        tt = 0
        for idx in range(8):
            bits = [(idx >> 2) & 1, (idx >> 1) & 1, idx & 1]  # v_bitop3: bit index a << 2 | b << 1 | c
            val = {}
            ok = True
            for l, bt in zip(leaves, bits):
                if l in val and val[l] != bt:
                    ok = False
                val.setdefault(l, bt)
            if ok and eval_cone(nodes, n, list(val), list(val.values())):
                tt |= 1 << idx
        gates.append((n, leaves, tt))
    return gates


def simulate(gates, x):
    v = {f"u{i}": (x >> (7 - i)) & 1 for i in range(8)}
    for n, (a, b, c), tt in gates:
        v[n] = (tt >> (v[a] << 2 | v[b] << 1 | v[c])) & 1
    return sum(v[f"s{i}"] << (7 - i) for i in range(8))


def emit(gates, path):
    lines = [
        "/* bs8_sbox.h -- GENERATED by tools/bs_probe/lut3_map.py: the Boyar-Peralta AES S-box (eprint 2009/191,",
        f" * 113 two-input gates) mapped onto {len(gates)} three-input gates (v_bitop3_b32; truth-table bit a << 2 | b << 1 | c).",
        " * The generator checks the mapped circuit on all 256 inputs; included by bs8_aes.h.  Do not edit by hand. */",
        "BS8_INL void sbox(uint32_t (&x)[8])",
        "{",
        "    const uint32_t u0 = x[7], u1 = x[6], u2 = x[5], u3 = x[4], u4 = x[3], u5 = x[2], u6 = x[1], u7 = x[0];",
    ]
    for n, (a, b, c), tt in gates:
        lines.append(f"    const uint32_t {n} = bitop3<0x{tt:02x}>({a}, {b}, {c});")
    lines.append("    x[7] = s0, x[6] = s1, x[5] = s2, x[4] = s3, x[3] = s4, x[2] = s5, x[1] = s6, x[0] = s7;")
    lines.append("}")
    open(path, "w").write("\n".join(lines) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "bs8_sbox.h"))
    args = ap.parse_args()
    nodes, order = parse()
    S = aes_sbox()
    cuts = enumerate_cuts(nodes, order)
    rng = random.Random(args.seed)
    best = None
    for it in range(args.iters):
        choice, need = map_circuit(nodes, order, cuts, rng)
        if best is None or len(need) < len(best[1]):
            best = (dict(choice), set(need))
            print(f"iter {it}: {len(need)} gates", file=sys.stderr)
    gates = topo_emit(nodes, order, best[0], best[1])
    bad = sum(simulate(gates, x) != S[x] for x in range(256))
    if bad:
        raise SystemExit(f"mapped S-box wrong on {bad} inputs")
    emit(gates, args.out)
    print(f"{len(gates)} gates -> {os.path.normpath(args.out)} (256/256 inputs checked)")


if __name__ == "__main__":
    main()

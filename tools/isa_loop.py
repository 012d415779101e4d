"""Instruction mix of the innermost loops of one kernel in a hipcc -S listing (gfx950).

Splits the kernel's code into basic blocks (labels, branches, fall-through), finds each natural loop
(blocks that reach a back edge to the loop header without passing the header) and prints the
instruction counts of every loop body -- e.g. the v_accvgpr copies, s_waitcnt vmcnt drains and
ds_read / MFMA counts of a staging loop.
usage: python tools/isa_loop.py <file.s> <kernel-symbol-substring> [top]
"""
import re
import sys
from collections import Counter


def kernel_lines(path, sym):
    out, on = [], False
    for ln in open(path):
        if not on and re.match(r"^_Z\S*" + re.escape(sym) + r"\S*:", ln):
            on = True
            continue
        if on:
            if ln.strip().startswith("s_endpgm"):
                out.append(ln)
                break
            out.append(ln)
    return out


def blocks(lines):
    bl, cur, name = [], [], "entry"
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            bl.append((name, cur))
            name, cur = m.group(1), []
            continue
        s = ln.split(";")[0].strip()
        if s:
            cur.append(s)
    bl.append((name, cur))
    return bl


def cfg(bl):
    succ = {}
    for i, (n, ins) in enumerate(bl):
        s = set()
        last = ins[-1] if ins else ""
        for x in ins:
            m = re.match(r"s_(c)?branch\S*\s+(\.LBB\S+)", x)
            if m:
                s.add(m.group(2))
        if not last.startswith("s_branch") and not last.startswith("s_endpgm") and i + 1 < len(bl):
            s.add(bl[i + 1][0])
        succ[n] = s
    return succ


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    bl = blocks(kernel_lines(path, sym))
    body = dict(bl)
    succ = cfg(bl)
    pred = {n: set() for n in body}
    for n, ss in succ.items():
        for t in ss:
            if t in pred:
                pred[t].add(n)
    order = [n for n, _ in bl]
    pos = {n: i for i, n in enumerate(order)}
    heads = [n for n, ins in bl if any(True for _ in [0]) and n in pred]
    loops = []
    for h in order:
        # back edges: predecessors dominated... approximated by a reachability test from h
        srcs = [p for p in pred[h] if reach(succ, h, p)]
        if not srcs:
            continue
        nodes = {h}
        stack = [p for p in srcs]
        while stack:
            x = stack.pop()
            if x in nodes:
                continue
            nodes.add(x)
            stack.extend(pred[x])
        loops.append((h, nodes))
    for h, nodes in loops:
        c = Counter()
        for n in nodes:
            for x in body[n]:
                c[x.split()[0]] += 1
        tot = sum(c.values())
        print(f"loop {h}: {len(nodes)} blocks, {tot} instructions; mfma {sum(v for k, v in c.items() if 'mfma' in k)}")
        for k, v in c.most_common(top):
            print(f"  {v:5d} {k}")
        waits = Counter(x for n in nodes for x in body[n] if x.startswith("s_waitcnt"))
        print("  waits:", dict(waits.most_common(8)))


def reach(succ, a, b):
    seen, stack = set(), [a]
    while stack:
        x = stack.pop()
        if x == b:
            return True
        if x in seen:
            continue
        seen.add(x)
        stack.extend(succ.get(x, ()))
    return False


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Static check of the hand-counted load rings in the GEMV kernels.

Inline-asm loads are invisible to hipcc's waitcnt bookkeeping, so a compiler-inserted copy of a
ring register between its asm load and the covering `s_waitcnt vmcnt` would read stale data.
This scans the device assembly of every kernel in a .s file: for each VGPR written by an asm
`global_load_*`, any instruction that reads it before the next `s_waitcnt vmcnt(...)` (which,
by construction of the ring, is the first wait that can cover it) is reported.
Usage: python tools/check_asm_ring.py file.s  (exit status 1 if a hazard is found)
"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def scan(body, seed):
    """One linear pass over a kernel. Outstanding vector-memory ops are an ordered queue (issue
    order); `s_waitcnt vmcnt(N)` retires all but the newest N. `seed` maps a loop label to the
    queue at its back-edge. Returns (hazards, queue-at-backedge per label)."""
    queue = []  # list of (set(regs) or empty, is_asm)
    in_asm = False
    hazards = []
    back = {}
    labels_seen = set()
    for i, line in enumerate(body):
        s = line.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        lm = re.match(r"^(\.LBB\w+):", s)
        if lm:
            labels_seen.add(lm.group(1))
            if lm.group(1) in seed:
                queue = list(seed[lm.group(1)]) + queue
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        args = [a.strip() for a in s[len(op):].split(",")]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = args[0].split()[0] if args else ""
            if tgt in labels_seen:
                back[tgt] = list(queue)
            continue
        if op.startswith("s_waitcnt") and "vmcnt" in s:
            n = int(re.search(r"vmcnt\((\d+)\)", s).group(1))
            while len(queue) > n:
                queue.pop(0)
            continue
        # reads of pending asm-load destinations
        if op.startswith("global_load") or op.startswith("buffer_load"):
            srcs = regs(args[1].split()[0]) if len(args) > 1 else set()
        elif op.startswith("global_store") or op.startswith("buffer_store"):
            srcs = set()
            for a in args[:2]:
                srcs |= regs(a.split()[0])
        else:
            srcs = set()
            for a in args[1:]:
                if a:
                    srcs |= regs(a.split()[0])
        pend = set()
        for r_, asm in queue:
            if asm:
                pend |= r_
        hit = srcs & pend
        if hit:
            hazards.append((i, s, sorted(hit)[0]))
        if op.startswith(("global_load", "buffer_load")):
            queue.append((regs(args[0]) if in_asm else set(), in_asm))
        elif op.startswith(("global_store", "buffer_store", "global_atomic", "buffer_atomic")):
            queue.append((set(), False))
    return hazards, back


def check(path):
    text = open(path).read()
    bad = 0
    for km in re.finditer(r"^(_Z\S+):", text, re.M):
        name = km.group(1)
        end = text.find(".Lfunc_end", km.end())
        body = text[km.end():end].split("\n")
        _, back = scan(body, {})
        hazards, _ = scan(body, back)
        for i, s, r in hazards:
            bad += 1
            print(f"{name[:90]}: line {i}: '{s}' reads asm-load dest v{r} before a vmcnt wait")
    return bad


if __name__ == "__main__":
    n = sum(check(p) for p in sys.argv[1:])
    print(f"{n} hazard(s)")
    sys.exit(1 if n else 0)

#!/usr/bin/env python3
"""Static check of the hand-counted load rings (inline-asm `global_load`s) in the decode kernels.

Inline-asm loads are invisible to hipcc's waitcnt bookkeeping, so any compiler-generated
instruction that touches an asm-load destination register (reads it, or writes it: the load's late
arrival would clobber the new value) before the `s_waitcnt vmcnt(N)` that retires that load is a
hazard (stale data / corrupted register). This scans the device assembly of every kernel:

  * outstanding vector-memory ops are an ordered queue (issue order); `s_waitcnt vmcnt(N)` retires
    all but the newest N (stores and atomics count too, as on CDNA4);
  * control flow: the state at a label is the union of the fall-through state and the states at
    every branch that targets it (forward branches in the same pass, back-edges from a first
    pass); code after an unconditional `s_branch` is only entered through its label.

Usage: python tools/check_asm_ring.py file.s   (exit status 1 if any hazard is found)
"""
import re
import sys

_VMEM = ("global_load", "buffer_load", "global_store", "buffer_store", "global_atomic", "buffer_atomic",
         "flat_load", "flat_store")


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _merge(a, b):
    """Union of two queues (pessimistic): keep the longer one's order, add missing asm entries."""
    if a is None:
        return None if b is None else list(b)
    if b is None:
        return list(a)
    out = list(a) if len(a) >= len(b) else list(b)
    other = b if out is a else a
    have = set()
    for r, asm in out:
        have |= r
    for r, asm in other:
        if asm and not (r <= have):
            out.insert(0, (r, asm))  # oldest position: retired first, i.e. least pessimistic
    return out


def scan(body, seed):
    queue = []           # list of (set(regs), is_asm); None = unreachable
    pending_in = {k: list(v) for k, v in seed.items()}
    in_asm = False
    hazards = []
    back = {}
    seen = set()
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
            lab = lm.group(1)
            seen.add(lab)
            queue = _merge(queue, pending_in.get(lab))
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        if queue is None:
            continue  # unreachable by fall-through
        op = s.split()[0]
        args = [a.strip() for a in s[len(op):].split(",")]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = args[0].split()[0] if args else ""
            if tgt in seen:
                back[tgt] = _merge(back.get(tgt), queue)
            else:
                pending_in[tgt] = _merge(pending_in.get(tgt), queue)
            if op == "s_branch":
                queue = None
            continue
        if op.startswith("s_waitcnt") and "vmcnt" in s:
            n = int(re.search(r"vmcnt\((\d+)\)", s).group(1))
            while len(queue) > n:
                queue.pop(0)
            continue
        if op.startswith("s_") or op.startswith("ds_"):
            touched = set()
            if op.startswith("ds_"):
                for a in args:
                    if a:
                        touched |= regs(a.split()[0])
        else:
            touched = set()
            for a in args:
                if a:
                    touched |= regs(a.split()[0])
            if op.startswith(_VMEM) and in_asm and "_lds" not in op:
                touched -= regs(args[0])  # the asm load's own destination (tied operand)
        pend = set()
        for r_, asm in queue:
            if asm:
                pend |= r_
        hit = touched & pend
        if hit:
            hazards.append((i, s, sorted(hit)[0]))
        if op.startswith(_VMEM):
            # global_load_lds_*: the first operand is the address (the data goes to LDS, no VGPR destination)
            is_load = "load" in op and "_lds" not in op
            queue.append((regs(args[0]) if (in_asm and is_load) else set(), in_asm and is_load))
    return hazards, back


def check(path):
    text = open(path).read()
    bad = 0
    for km in re.finditer(r"^(_Z\S+):", text, re.M):
        name = km.group(1)
        end = text.find(".Lfunc_end", km.end())
        if end < 0:
            continue
        body = text[km.end():end].split("\n")
        _, back = scan(body, {})
        hazards, _ = scan(body, back)
        for i, s, r in hazards:
            bad += 1
            print(f"{name[:90]}: line {i}: '{s}' touches asm-load dest v{r} before its vmcnt wait")
    return bad


if __name__ == "__main__":
    n = sum(check(p) for p in sys.argv[1:])
    print(f"{n} hazard(s)")
    sys.exit(1 if n else 0)

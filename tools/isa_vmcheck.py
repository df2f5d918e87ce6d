#!/usr/bin/env python3
"""Check the counted vector-memory waits of the conv tiles on their gfx950 ISA.

The LDS-DMA tiles (conv_winoc.hip, conv_winoh.hip, conv_block0.hip, ...) wait for a
staged tile with an inline-asm ``s_waitcnt vmcnt(N)``: everything but the N youngest
vector-memory loads must have returned.  N is fixed in the source, so it is right only
if the compiler emits the loads in the order the source assumed -- DESIGN.md §10: a
build with ``-amdgpu-sched-strategy=max-ilp`` moved U loads across a DMA issue group
and the kind-6 tile read LDS stages before they landed.

Every such wait is written with ``RRIN_VMWAIT(lds, ld)`` (common.hpp), whose asm text
carries the declaration ``; rrin-vm lds=A ld=B``: the N = A + B youngest loads before
the wait are A LDS-DMA pieces and B register loads.  This tool walks the control-flow
graph of every kernel in a ``hipcc --cuda-device-only -S`` listing backwards from each
declared wait, over every path, and checks that the N youngest vector-memory loads have
exactly that composition.  Loads return in issue order among themselves, so a matching
composition proves that every load issued before them -- the awaited DMA -- is done.
Stores are skipped: vmcnt counts them too, but they return out of order with loads, so
a younger store can only make the wait stricter, never let it pass early.

Fails (exit 1) on:
  * a declared wait whose youngest N loads differ from the declaration on some path
    (the compiler moved a load across the issue group the count relies on);
  * a path from the kernel entry with fewer than N loads before the wait;
  * an inline-asm ``s_waitcnt vmcnt(N > 0)`` without a declaration;
  * an atomic or a scratch (spill) load among the N youngest.

Usage:  isa_vmcheck.py FILE.s [FILE.s ...] [-v]
Run by ``make check-isa`` on the product sources (the CPU-side build check).
"""
import re
import sys
from collections import defaultdict

RE_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
RE_FUNC_TYPE = re.compile(r"^\s*\.type\s+([^,]+),@function")
RE_FUNC_END = re.compile(r"^\.Lfunc_end\d+:")
RE_DECL = re.compile(r"rrin-vm\s+lds=(\d+)\s+ld=(\d+)")
RE_VMCNT = re.compile(r"\bs_waitcnt\b.*\bvmcnt\((\d+)\)")

# vector-memory instruction classes (gfx950 = GFX9: vmcnt counts loads, LDS-DMA and stores)
def classify(ins):
    """'lds' LDS-DMA load, 'ld' load to registers, 'st' store, 'atomic', 'scratch' spill
    load, or None (not counted by vmcnt)."""
    m = ins.split(None, 1)
    if not m:
        return None
    op = m[0]
    rest = m[1] if len(m) > 1 else ""
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        if "atomic" in op:
            return "atomic"
        if "_store" in op:
            return "st"
        if "_load" in op:
            if op.startswith("scratch_"):
                return "scratch"
            # buffer_load_* ... lds  /  global_load_lds_dwordx*
            if re.search(r"\blds\b", rest) or op.startswith("global_load_lds"):
                return "lds"
            return "ld"
        if op.startswith("buffer_wbl2") or op.startswith("buffer_inv") or op.startswith("buffer_gl"):
            return None
    return None


class Func:
    def __init__(self, name):
        self.name = name
        self.blocks = []  # [label, [ (lineno, text, in_asm) ]]
        self.succ = defaultdict(list)


def parse(path):
    funcs = []
    fn_names = set()
    cur = None
    in_asm = False
    with open(path) as f:
        lines = f.read().split("\n")
    for no, raw in enumerate(lines, 1):
        m = RE_FUNC_TYPE.match(raw)
        if m:
            fn_names.add(m.group(1).strip())
            continue
        s = raw.strip()
        if cur is None:
            s = s.split(";", 1)[0].strip()
            if s.endswith(":") and s[:-1] in fn_names:
                cur = Func(s[:-1])
                cur.blocks.append(["<entry>", []])
                in_asm = False
            continue
        if RE_FUNC_END.match(s):
            funcs.append(cur)
            cur = None
            continue
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = RE_LABEL.match(s)
        if m:
            cur.blocks.append([m.group(1), []])
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.blocks[-1][1].append((no, s, in_asm))
    return funcs


def build_cfg(fn):
    labels = {b[0]: i for i, b in enumerate(fn.blocks)}
    preds = defaultdict(list)
    for i, (lab, ins) in enumerate(fn.blocks):
        falls = True
        for (_, s, _) in ins:
            op = s.split()[0]
            if op == "s_branch":
                tgt = s.split()[1]
                preds[labels[tgt]].append(i)
                falls = False
            elif op.startswith("s_cbranch"):
                tgt = s.split()[1]
                preds[labels[tgt]].append(i)
            elif op in ("s_endpgm", "s_setpc_b64", "s_trap"):
                falls = False
        if falls and i + 1 < len(fn.blocks):
            preds[i + 1].append(i)
    return preds


def check_wait(fn, preds, bi, ii, n, want, errors, verbose):
    """Backward DFS over every path from instruction ii of block bi."""
    seen = set()
    results = set()
    stack = [(bi, ii, ())]  # found: tuple of classes, youngest first
    while stack:
        b, i, found = stack.pop()
        ins = fn.blocks[b][1]
        done = False
        for k in range(i - 1, -1, -1):
            c = classify(ins[k][1])
            if c is None or c == "st":
                continue
            found = found + ((c, ins[k][0]),)
            if len(found) == n:
                done = True
                break
        if done:
            comp = {"lds": 0, "ld": 0}
            bad = [f"{c}@{ln}" for (c, ln) in found if c not in comp]
            for (c, _) in found:
                if c in comp:
                    comp[c] += 1
            key = (comp["lds"], comp["ld"], tuple(bad))
            if key not in results:
                results.add(key)
                if bad or (comp["lds"], comp["ld"]) != want:
                    errors.append(
                        f"  youngest {n} loads on a path: lds={comp['lds']} ld={comp['ld']}"
                        + (f" other={bad}" if bad else "")
                        + f" (declared lds={want[0]} ld={want[1]}); loads at lines "
                        + ",".join(str(ln) for (_, ln) in found)
                    )
            continue
        if not preds.get(b):
            errors.append(f"  a path from the kernel entry has only {len(found)} of {n} loads before the wait")
            continue
        for p in preds[b]:
            st = (p, tuple(c for (c, _) in found))
            if st in seen:
                continue
            seen.add(st)
            stack.append((p, len(fn.blocks[p][1]), found))
    return results


def check_file(path, verbose=False):
    nwaits = 0
    failures = 0
    for fn in parse(path):
        preds = build_cfg(fn)
        for bi, (lab, ins) in enumerate(fn.blocks):
            for ii, (no, s, in_asm) in enumerate(ins):
                m = RE_VMCNT.search(s)
                if not m or not in_asm:
                    continue
                n = int(m.group(1))
                d = RE_DECL.search(s)
                if n == 0:
                    continue
                errors = []
                if not d:
                    errors.append("  counted inline-asm wait without an rrin-vm declaration (use RRIN_VMWAIT)")
                    res = set()
                else:
                    want = (int(d.group(1)), int(d.group(2)))
                    if sum(want) != n:
                        errors.append(f"  declaration lds+ld = {sum(want)} != vmcnt({n})")
                    res = check_wait(fn, preds, bi, ii, n, want, errors, verbose)
                nwaits += 1
                if errors:
                    failures += 1
                    print(f"FAIL {path}:{no} {fn.name}: {s}")
                    for e in errors:
                        print(e)
                elif verbose:
                    print(f"ok   {path}:{no} {fn.name}: vmcnt({n}) paths {sorted(res)}")
    return nwaits, failures


def main(argv):
    verbose = "-v" in argv
    files = [a for a in argv if a != "-v"]
    if not files:
        print(__doc__)
        return 2
    total = fail = 0
    for f in files:
        n, k = check_file(f, verbose)
        total += n
        fail += k
        print(f"{f}: {n} counted waits checked, {k} failed")
    return 1 if fail else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

"""Audit of the inline-asm vector loads in a kernel's ISA (VERDICT r5 "Next round" 1: hand-managed waits).

hipcc does not know that an inline-asm ``global_load_*`` writes its destination VGPRs LATER, when the data returns;
it only sees the asm statement define them.  Such a load is safe only if no instruction touches those registers
before an ``s_waitcnt vmcnt(n)`` retires it (n = the VMEM operations issued after it).  A register-allocator copy,
spill or reuse in that window reads / clobbers a register the load has not written yet: a timing-dependent bug.

This script splits each kernel into basic blocks, propagates over the control-flow graph (loops to a fixed point)
the inline-asm loads still outstanding with the count of VMEM operations issued after each, retires them at every
``s_waitcnt vmcnt(n)`` and reports every instruction that reads or writes a destination register of an outstanding
inline-asm load.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -Iinclude csrc/pz_flash.hip -o /tmp/pz_flash.s
    python tools/asm_async_audit.py /tmp/pz_flash.s [kernel-substring ...]
"""

from __future__ import annotations

import re
import sys

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
VMEM = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)(load|store|atomic)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            out.update((m.group(3), r) for r in range(int(m.group(4)), int(m.group(5)) + 1))
    return out


def _blocks(lines):
    """basic blocks [(label, [(line no, text, in_asm)])] and successor labels (fall-through + branch targets)"""
    blocks, cur, in_asm = [], ["<entry>", []], False
    blocks.append(cur)
    for no, raw in lines:
        if ";;#ASMSTART" in raw:
            in_asm = True
            continue
        if ";;#ASMEND" in raw:
            in_asm = False
            continue
        s = raw.split(";")[0].strip()
        lab = re.match(r"^(\.?L\w+|\S+):", s)
        if lab and not s.startswith("."):
            lab = None
        if lab or (not s and "%bb." in raw):
            name = lab.group(1) if lab else raw.strip().split()[1].rstrip(":")
            cur = [name, []]
            blocks.append(cur)
            continue
        if not s or s.startswith("."):
            continue
        cur[1].append((no, s, in_asm))
    succ = {}
    for i, (name, ins) in enumerate(blocks):
        out = []
        last = ins[-1][1] if ins else ""
        for _, s, _ in ins:
            m = re.match(r"s_(c?branch\w*)\s+(\S+)", s)
            if m:
                out.append(m.group(2))
        if not last.startswith(("s_branch", "s_endpgm", "s_setpc")) and i + 1 < len(blocks):
            out.append(blocks[i + 1][0])
        succ[name] = out
    return blocks, succ


def audit(lines, name):
    """dataflow over the CFG: state = {inline load id: (dest regs, VMEM ops issued after it)}, joined by keeping a
    load pending if it is pending on any incoming path (with the smaller count)"""
    blocks, succ = _blocks(lines)
    bmap = {b[0]: b[1] for b in blocks}
    loads = {}
    state_in = {blocks[0][0]: {}}
    work = [blocks[0][0]]
    issues = {}
    while work:
        bname = work.pop()
        st = dict(state_in.get(bname, {}))
        for no, s, in_asm in bmap.get(bname, []):
            m = re.match(r"s_waitcnt\b(.*)", s)
            if m:
                vm = re.search(r"vmcnt\((\d+)\)", m.group(1))
                if vm:
                    k = int(vm.group(1))
                    st = {i: v for i, v in st.items() if v[1] < k}
                continue
            if VMEM.match(s):
                op, _, rest = s.partition(" ")
                ops = [o.strip() for o in rest.split(",")]
                # loads, and atomics that return the old value (sc0 / glc), write a destination register
                is_load = ("load" in op and "lds" not in op) or ("atomic" in op and re.search(r"\b(sc0|glc)\b", rest))
                rd = regs(",".join(ops[1:])) if is_load else regs(rest)
                for i, (d, _) in st.items():
                    if rd & d:
                        issues[(no, i)] = s
                st = {i: (d, min(c + 1, 64)) for i, (d, c) in st.items()}
                if in_asm and is_load:
                    loads[no] = s
                    st[no] = (regs(ops[0]), 0)
                continue
            t = regs(s)
            for i, (d, _) in st.items():
                if t & d:
                    issues[(no, i)] = s
        for nb in succ.get(bname, []):
            if nb not in bmap:
                continue
            old = state_in.get(nb)
            if old is None:
                state_in[nb] = dict(st)
                work.append(nb)
                continue
            merged = dict(old)
            for i, v in st.items():
                merged[i] = v if i not in merged else (v[0], min(v[1], merged[i][1]))
            if merged != old:
                state_in[nb] = merged
                work.append(nb)
    print(f"{name}: {len(loads)} inline-asm VMEM loads, {len(issues)} touches before their vmcnt")
    for (no, i), s in sorted(issues.items())[:40]:
        print(f"    line {no}: {s}\n        touches the destination of line {i}: {loads[i]}")
    return issues


def main():
    path = sys.argv[1]
    want = sys.argv[2:]
    text = open(path).read().splitlines()
    kernels = []
    cur = None
    for i, line in enumerate(text, 1):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = (m.group(1), [])
            kernels.append(cur)
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            cur[1].append((i, line))
    bad = 0
    for name, body in kernels:
        if want and not any(w in name for w in want):
            continue
        if not any("ASMSTART" in l for _, l in body):
            continue
        bad += len(audit(body, name))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Check the vmcnt waits of compiler-emitted gfx950 assembly against its VMEM loads, path by path.

Abstract interpretation over the kernel's control-flow graph, with the hardware's in-order counter
semantics: every vector-memory instruction (buffer / global / scratch loads and stores, and the
global_load_lds DMA loads inside inline asm, which the compiler's waitcnt pass does not see) is one
vmcnt event; `s_waitcnt vmcnt(N)` retires all but the newest N.  State per program point: for each VGPR
with a load still possibly in flight, the fewest events issued after that load on any path.  An
instruction that reads or overwrites such a VGPR is reported: on that path the data may not have
landed.  Both counting models are checked: --asm-vmem 1 counts the asm DMA loads as the hardware
does, 0 as the compiler's pass does.

  python3 tools/vmcnt_check.py /tmp/isa/kernel.s [--kernel SUBSTR] [--asm-vmem 0|1]
"""
import argparse
import re

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(path, want):
    lines = open(path).read().splitlines()
    kern, body, in_asm = None, [], False
    for raw in lines:
        s = raw.strip()
        if re.match(r"^_Z\w+:", s) and not raw[:1].isspace():
            if kern and want in kern:
                break
            kern, body = s.split(":")[0], []
            continue
        if kern is None:
            continue
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(\.LBB\w+):", s) or re.match(r"^; %(bb\.\d+):", s)
        if m:
            body.append(("label", m.group(1)))
            continue
        if not s or s[0] in ";." or s.endswith(":"):
            continue
        body.append(("inst", s.split(";")[0].strip(), in_asm))
        if s.startswith("s_endpgm"):
            pass
    return kern, body


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--asm-vmem", type=int, default=1)
    args = ap.parse_args()
    kern, body = parse(args.path, args.kernel)
    # basic blocks
    blocks, cur, labels = [], None, {}
    for it in body:
        if it[0] == "label":
            cur = {"label": it[1], "insts": [], "succ": []}
            labels[it[1]] = len(blocks)
            blocks.append(cur)
            continue
        if cur is None:
            cur = {"label": "entry", "insts": [], "succ": []}
            blocks.append(cur)
        cur["insts"].append(it)
        if re.match(r"^s_(branch|cbranch_\w+|endpgm)\b", it[1]):
            cur = {"label": f"after{len(blocks)}", "insts": [], "succ": []}
            blocks.append(cur)
    for i, b in enumerate(blocks):
        last = b["insts"][-1][1] if b["insts"] else ""
        mn = last.split()[0] if last else ""
        if mn.startswith("s_cbranch") or mn == "s_branch":
            tgt = last.split()[1]
            if tgt in labels:
                b["succ"].append(labels[tgt])
        if mn not in ("s_branch", "s_endpgm") and i + 1 < len(blocks):
            b["succ"].append(i + 1)

    CAP = 64

    def is_vmem(m):
        return re.match(r"^(buffer|global|scratch)_(load|store|atomic)", m) is not None

    def transfer(state, b, report):
        st = dict(state)
        for _, text, in_asm in b["insts"]:
            m = text.split()[0]
            ops = text[len(m):]
            if m == "s_waitcnt" and "vmcnt(" in text:
                n = int(re.search(r"vmcnt\((\d+)\)", text).group(1))
                st = {r: c for r, c in st.items() if c < n}
                continue
            if is_vmem(m) and (args.asm_vmem or not in_asm):
                fields = [f.strip() for f in ops.split(",")]
                srcs = set()
                if "_load" in m and "_lds" not in m:
                    dst = regs(fields[0])
                    srcs = set().union(*[regs(f) for f in fields[1:]]) if len(fields) > 1 else set()
                else:
                    dst = set()
                    srcs = regs(ops)
                for r in (srcs | dst) & set(st):
                    report.append((b["label"], text, r, st[r]))
                st = {r: min(c + 1, CAP) for r, c in st.items()}
                for r in dst:
                    st[r] = 0
                continue
            if m.startswith("v_") or m.startswith("ds_") or m.startswith("s_") and "v" in ops:
                used = regs(ops)
                for r in used & set(st):
                    report.append((b["label"], text, r, st[r]))
        return st

    IN = [None] * len(blocks)
    IN[0] = {}
    work = [0]
    it = 0
    while work and it < 20000:
        it += 1
        i = work.pop(0)
        out = transfer(IN[i], blocks[i], [])
        for s in blocks[i]["succ"]:
            if IN[s] is None:
                new = dict(out)
            else:
                new = dict(IN[s])
                for r, c in out.items():
                    new[r] = min(new.get(r, CAP), c)
            if new != IN[s]:
                IN[s] = new
                work.append(s)
    reports = []
    for i, b in enumerate(blocks):
        if IN[i] is not None:
            transfer(IN[i], b, reports)
    seen = set()
    print(f"kernel {kern}: {len(blocks)} blocks; asm DMA counted: {bool(args.asm_vmem)}")
    for lab, text, r, c in reports:
        key = (lab, text, r)
        if key in seen:
            continue
        seen.add(key)
        print(f"  {lab}: v{r} read/written with its load possibly in flight ({c} events issued after it): {text}")
    if not reports:
        print("  no unguarded use of an in-flight load")


if __name__ == "__main__":
    main()

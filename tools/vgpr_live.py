"""Rough VGPR liveness over a kernel's gfx9 assembly (hipcc -S): where the
register peak of a kernel is and which source lines hold it.

    python tools/vgpr_live.py file.s KERNEL_SUBSTRING [--top N]

Backward dataflow over the basic blocks of the listing (labels and branches),
defs and uses read off the operand lists.  A def under a partial exec mask
does not end a lane's value in reality, so the numbers are a lower bound near
divergent code; good enough to find the region that sets the peak.
"""
import re
import sys
from collections import defaultdict

STORE = re.compile(r"^(global_store|buffer_store|flat_store|scratch_store|ds_write|ds_store|ds_add|ds_max|ds_min|"
                   r"global_atomic(?!.*glc)|s_|v_cmp|v_cmpx|v_readlane|v_readfirstlane|ds_swizzle_b32_nodef)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = []
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.append(int(m.group(3)))
        else:
            out.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(lines):
    ins = []  # (label or None, mnemonic, defs, uses, raw, loc)
    loc = ""
    for raw in lines:
        t = raw.strip()
        if t.startswith(".loc"):
            parts = t.split()
            loc = f"{parts[1]}:{parts[2]}"
            continue
        if not t or t.startswith(";") or (t.startswith(".") and not t.endswith(":")):
            continue
        if t.endswith(":"):
            ins.append((t[:-1], None, [], [], t, loc))
            continue
        t = t.split(";")[0].strip()
        mn, _, ops = t.partition(" ")
        opl = [o.strip() for o in ops.split(",")] if ops else []
        if not opl:
            ins.append((None, mn, [], [], t, loc))
            continue
        if STORE.match(mn):
            defs, uses = [], regs(ops)
            if mn.startswith("v_writelane"):
                defs = regs(opl[0])
        else:
            defs, uses = regs(opl[0]), regs(",".join(opl[1:]))
            if mn.startswith("v_writelane") or mn.startswith("v_mov_b32_dpp") or "_dpp" in mn:
                uses += defs  # partial writes
        ins.append((None, mn, defs, uses, t, loc))
    return ins


def analyse(ins):
    # basic blocks
    starts = [0] + [i for i, x in enumerate(ins) if x[0] is not None]
    for i, x in enumerate(ins):
        if x[1] and (x[1].startswith("s_branch") or x[1].startswith("s_cbranch") or x[1] in ("s_endpgm",)):
            starts.append(i + 1)
    starts = sorted(set(s for s in starts if s < len(ins)))
    blocks = [(s, e) for s, e in zip(starts, starts[1:] + [len(ins)])]
    label_block = {}
    for bi, (s, e) in enumerate(blocks):
        if ins[s][0] is not None:
            label_block[ins[s][0]] = bi
    succ = defaultdict(list)
    for bi, (s, e) in enumerate(blocks):
        last = ins[e - 1]
        mn = last[1] or ""
        if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            tgt = last[4].split()[-1]
            if tgt in label_block:
                succ[bi].append(label_block[tgt])
            if mn.startswith("s_cbranch") and bi + 1 < len(blocks):
                succ[bi].append(bi + 1)
        elif mn != "s_endpgm" and bi + 1 < len(blocks):
            succ[bi].append(bi + 1)
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for bi in range(len(blocks) - 1, -1, -1):
            s, e = blocks[bi]
            live = set().union(*[live_in[t] for t in succ[bi]]) if succ[bi] else set()
            for i in range(e - 1, s - 1, -1):
                live -= set(ins[i][2])
                live |= set(ins[i][3])
            if live != live_in[bi]:
                live_in[bi] = live
                changed = True
    # pressure at every instruction
    press = [0] * len(ins)
    for bi, (s, e) in enumerate(blocks):
        live = set().union(*[live_in[t] for t in succ[bi]]) if succ[bi] else set()
        for i in range(e - 1, s - 1, -1):
            live -= set(ins[i][2])
            live |= set(ins[i][3])
            press[i] = len(live | set(ins[i][2]))
    return press


def main():
    path, kern = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    text = open(path).read()
    names = re.findall(r"^(\S*" + re.escape(kern) + r"\S*):", text, re.M)
    if not names:
        sys.exit("kernel not found")
    name = names[0]
    i = text.index(name + ":")
    j = text.index(".Lfunc_end", i)
    ins = parse(text[i:j].splitlines()[1:])
    press = analyse(ins)
    print(name, "instructions", sum(1 for x in ins if x[1]), "max live VGPRs", max(press))
    by_loc = defaultdict(int)
    for x, p in zip(ins, press):
        by_loc[x[5]] = max(by_loc[x[5]], p)
    for loc, p in sorted(by_loc.items(), key=lambda kv: -kv[1])[:top]:
        print(f"  {p:4d}  {loc}")


if __name__ == "__main__":
    main()

"""Per-basic-block instruction mix of one kernel in a device assembly file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S \
        -I include -I nem-mcmc-optimization_amd/csrc <file>.hip -o k.s
    python tools/isa_blocks.py k.s <substring of the mangled kernel name>

Prints, per block, the VALU count split into the issue classes measured by
tools/ubench/valu_rate2.hip (VOP2-class ~2.5 cycles, VOP3 / f64 ~4.5), MFMAs,
DS and VMEM instructions -- enough to price a loop body before a GPU run.
"""
import re
import sys

# full-rate (VOP1/VOP2 encodings of 32-bit integer and move ops)
FULL = re.compile(r"^v_(mov_b32|and_b32|or_b32|xor_b32|lshrrev_b32|ashrrev_i32|lshlrev_b32|"
                  r"add_u32|sub_u32|subrev_u32|add_co_u32|sub_co_u32|addc_co_u32|cndmask_b32|"
                  r"not_b32|readfirstlane_b32|add_f32|mul_f32|fmac_f32|fma_f32|max_f32|min_f32)(_e32)?$")


def blocks(path, name):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(name) + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    out, cur = [], ["entry", []]
    out.append(cur)
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = [m.group(1), []]
            out.append(cur)
            continue
        t = l.strip()
        if t and not t.startswith(";") and not t.startswith("."):
            cur[1].append(t)
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    tot = {}
    for label, ins in blocks(path, name):
        ops = [i.split()[0] for i in ins]
        c = {
            "valu_full": sum(1 for o in ops if FULL.match(o)),
            "valu_other": sum(1 for o in ops if o.startswith("v_") and not o.startswith("v_mfma") and not FULL.match(o)),
            "mfma": sum(1 for o in ops if o.startswith("v_mfma")),
            "ds": sum(1 for o in ops if o.startswith("ds_")),
            "vmem": sum(1 for o in ops if o.startswith(("global_", "buffer_", "flat_"))),
            "salu": sum(1 for o in ops if o.startswith("s_")),
        }
        est = 2.5 * c["valu_full"] + 4.5 * c["valu_other"]
        print(f"{label:14s} n={len(ops):4d} " + " ".join(f"{k}={v}" for k, v in c.items()) + f" valu_cyc~{est:.0f}")
        if "-v" in sys.argv:
            from collections import Counter
            print("   ", Counter(o for o in ops if o.startswith("v_")).most_common(40))


if __name__ == "__main__":
    main()

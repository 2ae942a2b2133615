"""Instruction mix of the fused group-by kernel variants from the gfx950
device assembly (hipcc --cuda-device-only -S):

    hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \\
          -x hip --cuda-device-only -S polaroid_amd/csrc/groupby.hip -o /tmp/groupby_gfx950.s
    python tools/isa_stats.py /tmp/groupby_gfx950.s

For each variant: VGPRs / SGPRs / occupancy from the compiler's comments,
the whole kernel's instruction counts, and the basic blocks that issue the
per-row LDS atomics (ds_add_u64 / ds_add_rtn_u64), with their LDS,
s_waitcnt and VALU counts -- the per-selected-row work.
"""
import re
import sys

VARIANTS = {
    "headline 4 sums (SUMONLY, 2 limbs)": "ILi4ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi0ELi0ELb0EE",
    "vwap DERIV 2 accs": "ILi2ELi1ELb1ELi2ELi2ELb0ELb0ELb1ELi0ELi0EE",
    "vwap product pair (VAR 2)": "ILi2ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi2ELi0EE",
    "vwap-like 2 plain sums": "ILi2ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi0ELi0EE",
    "std VAR triple": "ILi3ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi1ELi0EE",
    "std VAR triple, x >= 0 (VAR 4)": "ILi3ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi4ELi0EE",
    "headline, close >= 0 (VAR 5)": "ILi4ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi5ELi0ELb0EE",
    "headline PACK (fused integer keys)": "ILi4ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi0ELi1EE",
    "headline PACK 1, close >= 0 (VAR 5)": "ILi4ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi5ELi1EE",
    "headline PACK (String key codes)": "ILi4ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi0ELi2EE",
    "headline NULLS (validity bitmaps)": "ILi4ELi1ELb1ELi2ELi2ELb0ELb0ELb0ELi0ELi0ELb1EE",
}


def blocks(body):
    cur, name = [], "entry"
    for line in body.split("\n"):
        if re.match(r"^\.LBB\S+:", line):
            yield name, cur
            name, cur = line.split(":")[0], []
        elif line.startswith("\t") and not line.strip().startswith((".", ";")):
            cur.append(line.strip())
    yield name, cur


def count(ins, prefix):
    return sum(1 for x in ins if x.startswith(prefix))


def main():
    s = open(sys.argv[1]).read()
    for title, tmpl in VARIANTS.items():
        sym = f"_ZN5plgpu14gb_fast_kernel{tmpl}EvNS_8GbParamsENS_10DevProgramE"
        i = s.find(f"\n{sym}:")
        if i < 0:
            print(f"{title}: not instantiated")
            continue
        j = s.index(".Lfunc_end", i)
        body = s[i:j]
        meta = s[j:j + 6000]
        def m(k):
            r = re.search(rf"; {k}: (\d+)", meta)
            return r.group(1) if r else "?"
        ins = [x for _, b in blocks(body) for x in b]
        print(f"== {title}: VGPRs {m('NumVgprs')} SGPRs {m('NumSgprs')} occupancy {m('Occupancy')} "
              f"waves/SIMD; {len(ins)} instructions, ds {count(ins, 'ds_')}, global_load "
              f"{count(ins, 'global_load')}, s_waitcnt {count(ins, 's_waitcnt')}")
        for name, b in blocks(body):
            at = count(b, "ds_add_u64") + count(b, "ds_add_rtn_u64")
            if at:
                print(f"   {name:10s} {len(b):4d} instr: ds_add {at}, ds_read {count(b, 'ds_read')}, "
                      f"s_waitcnt {count(b, 's_waitcnt')} (lgkmcnt {sum('lgkmcnt' in x for x in b)}), "
                      f"v_ {count(b, 'v_')}, s_ {count(b, 's_')}")


if __name__ == "__main__":
    main()

"""Instruction mix and register use of one kernel in a gfx950 assembly listing.

    hipcc --offload-arch=gfx950 <flags> --cuda-device-only -S x.hip -o /tmp/x.s
    python tools/isa_stats.py /tmp/x.s k_score [--dump]
"""
import collections
import re
import sys


def main(path, name, dump=False):
    s = open(path).read()
    for m in re.finditer(r"^(_Z\w*" + re.escape(name) + r"\w*):", s, re.M):
        sym = m.group(1)
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        ins = [ln.strip() for ln in body.split("\n")
               if ln.strip() and not ln.strip().startswith((".", ";", "//")) and not ln.strip().endswith(":")]
        c = collections.Counter(i.split()[0] for i in ins)
        meta = s[end:end + 4000]
        regs = dict(re.findall(r"\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):\s*(\d+)", s[s.find(sym, end):][:200000])[:4])
        kinds = collections.Counter()
        for k, v in c.items():
            kinds["valu" if k.startswith("v_") else "salu" if k.startswith("s_") and not k.startswith(("s_load", "s_waitcnt", "s_buffer")) else
                  "smem" if k.startswith(("s_load", "s_buffer")) else "vmem" if k.startswith(("global_", "buffer_", "flat_")) else
                  "lds" if k.startswith("ds_") else "wait" if k.startswith("s_waitcnt") else "other"] += v
        print(sym[:60], len(ins), dict(kinds), regs)
        print("  ", c.most_common(30))
        if dump:
            print("\n".join(ins))
        del meta


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "--dump" in sys.argv)

"""Dev tool: per-basic-block instruction mix of one kernel in a hipcc -S output.

usage: python tools/isa_blocks.py <file.s> <kernel-symbol-substring> [min_exp]
Prints the blocks that contain at least `min_exp` v_exp_f32 (the recurrence
bodies), with their VALU / SALU / LDS / VMEM counts and back-edge targets.
"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
min_exp = int(sys.argv[3]) if len(sys.argv) > 3 else 1
s = open(path).read()
m = re.search(r"^(\S*%s\S*):" % re.escape(name), s, re.M)
i = m.start()
j = s.index(".Lfunc_end", i)
blocks, cur, lab = [], [], "entry"
for line in s[i:j].split("\n"):
    t = line.split(";")[0].strip()
    if not t or t.startswith("."):
        if t.endswith(":"):
            blocks.append((lab, cur))
            lab, cur = t, []
        continue
    if t.endswith(":"):
        blocks.append((lab, cur))
        lab, cur = t, []
    else:
        cur.append(t)
blocks.append((lab, cur))
for lab, ins in blocks:
    ops = [x.split()[0] for x in ins]
    c = collections.Counter(ops)
    if c["v_exp_f32_e32"] + c["v_exp_f32_e64"] < min_exp:
        continue
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith(("v_readlane", "v_writelane")))
    salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_load", "s_buffer", "s_waitcnt",
                                                                                      "s_cbranch", "s_branch")))
    lds = sum(v for k, v in c.items() if k.startswith("ds_"))
    vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_")))
    smem = sum(v for k, v in c.items() if k.startswith(("s_load", "s_buffer_load")))
    br = [x for x in ins if x.startswith("s_cbranch") or x.startswith("s_branch")]
    print(f"{lab} n={len(ins)} valu={valu} salu={salu} lds={lds} vmem={vmem} smem={smem} "
          f"exp={c['v_exp_f32_e32'] + c['v_exp_f32_e64']} waitcnt={c['s_waitcnt']} branches={br}")
    print("   ", dict(c.most_common(18)))

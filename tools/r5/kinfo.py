"""Per-kernel resource summary from a -save-temps gfx950 .s file: VGPR / AGPR / LDS / scratch
and counts of chosen instructions.   python tools/r5/kinfo.py file.s PATTERN [insn ...]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
insns = sys.argv[3:] or ["v_mfma", "ds_read", "ds_write", "ds_add", "s_waitcnt", "v_cndmask"]
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    name = m.group(1)
    if not re.search(pat, name):
        continue
    end = s.find(".Lfunc_end", m.start())
    body = s[m.start():end]
    k = s.find(".amdhsa_kernel " + name)
    meta = s[k:s.find(".end_amdhsa_kernel", k)]

    def f(key):
        mm = re.search(r"\.amdhsa_" + key + r"\s+(\d+)", meta)
        return mm.group(1) if mm else "?"

    lead = r"^\s*"
    cnt = " ".join("%s=%d" % (i, len(re.findall(lead + i, body, re.M))) for i in insns)
    print(f"{name[:70]:70s} vgpr={f('next_free_vgpr')} acc_off={f('accum_offset')} lds={f('group_segment_fixed_size')} "
          f"scratch={f('private_segment_fixed_size')} {cnt}")

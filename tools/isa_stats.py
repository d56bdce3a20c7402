"""ISA statistics of kernels in a hipcc -save-temps .s file (dev tool): registers, spills,
waits, LDS-DMA copies and MFMAs per kernel whose name matches a pattern.

    python tools/isa_stats.py <file.s> <name-substring>
"""
import re
import sys


def main(path, pat):
    s = open(path).read()
    for m in re.finditer(r"^(\S*" + re.escape(pat) + r"\S*):\s*;", s, re.M):
        name = m.group(1)
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        meta = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"(.*?)\.end_amdhsa_kernel", s, re.S)
        info = {}
        if meta:
            for k in ("next_free_vgpr", "next_free_sgpr", "accum_offset", "private_segment_fixed_size",
                      "group_segment_fixed_size"):
                mm = re.search(r"\.amdhsa_" + k + r"\s+(\d+)", meta.group(1))
                info[k] = int(mm.group(1)) if mm else None
        cnt = {k: len(re.findall(p, body)) for k, p in (
            ("vmcnt_waits", r"s_waitcnt vmcnt"), ("vmcnt0", r"s_waitcnt vmcnt\(0\)"), ("glds", r"global_load_lds"),
            ("mfma", r"v_mfma"), ("scratch", r"scratch_"), ("ds_read", r"ds_read"), ("s_barrier", r"s_barrier"))}
        print(name[:80], info, cnt)


if __name__ == "__main__":
    main(*sys.argv[1:])

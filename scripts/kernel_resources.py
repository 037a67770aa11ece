"""Register / spill / LDS summary of kernels in a hipcc --cuda-device-only -S assembly file.

usage: python scripts/kernel_resources.py <file.s> [name-substring ...]
Parses the .amdgpu_metadata YAML (one '- .agpr_count' entry per kernel) and counts VALU / MFMA /
spill-related instructions in each kernel body."""
import collections
import re
import sys


def main(path, subs):
    s = open(path).read()
    meta = s[s.index("amdhsa.kernels:"):]
    entries = re.split(r"\n  - \.", meta)
    for e in entries[1:]:
        e = "." + e
        name = re.search(r"\.name:\s+(\S+)", e).group(1)
        if subs and not any(x in name for x in subs):
            continue
        f = {k: (re.search(r"\." + k + r":\s+(\d+)", e) or [None, "?"])[1] for k in
             ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
              "private_segment_fixed_size", "group_segment_fixed_size")}
        i = s.find(name + ":")
        j = s.find("s_endpgm", i)
        c = collections.Counter(m.group(1) for m in re.finditer(r"\n\s+([vsdgb][a-z0-9_]+)", s[i:j]))
        valu = sum(n for k, n in c.items() if k.startswith("v_") and "mfma" not in k)
        mfma = sum(n for k, n in c.items() if "mfma" in k)
        print(f"{name[:90]}\n   {f}\n   static: VALU {valu} MFMA {mfma} readlane {c['v_readlane_b32']} "
              f"writelane {c['v_writelane_b32']} accvgpr_read {c['v_accvgpr_read_b32']} "
              f"scratch {c['scratch_load_dword'] + c['scratch_store_dword'] + c['scratch_load_dwordx2'] + c['scratch_store_dwordx2'] + c['scratch_load_dwordx4'] + c['scratch_store_dwordx4']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])

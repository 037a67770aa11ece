"""LDS fragment-read pipelining in a compiled kernel: for every ds_read_b128 whose destination quad
is an operand of a later v_mfma_f32_16x16x32_f16, the number of MFMAs issued between the read and
that first consumer (0-2: read, waited on and multiplied in turn; >= 6: read a 6-MFMA group ahead).

usage: hipcc ... --cuda-device-only -S rlp_update.hip -o upd.s
       python scripts/isa_read_gaps.py upd.s <mangled kernel name> [...]
(FD fragment-read pipelining.)"""
import collections
import re
import sys


def gaps(asm, name):
    i = asm.find(name + ":")
    j = asm.find("s_endpgm", i)
    pend, out = {}, []
    for line in asm[i:j].split("\n"):
        line = line.strip()
        m = re.match(r"ds_read_b128 v\[(\d+):\d+\]", line)
        if m:
            pend[int(m.group(1))] = 0
            continue
        if line.startswith("v_mfma_f32_16x16x32_f16"):
            ops = [o.strip() for o in line.split(None, 1)[1].split(",")]
            srcs = [int(m.group(1)) for m in (re.match(r"v\[(\d+):\d+\]", o) for o in ops[1:3]) if m]
            for r in list(pend):
                if r in srcs:
                    out.append(pend.pop(r))
            for r in pend:
                pend[r] += 1
    return out


def main(path, names):
    asm = open(path).read()
    for name in names:
        g = gaps(asm, name)
        c = collections.Counter(min(x, 6) for x in g)
        print(f"{name[:60]}: {len(g)} reads consumed, gap <= 2: "
              f"{sum(v for k, v in c.items() if k <= 2)}, gap >= 6: {c[6]}  {dict(sorted(c.items()))}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])

"""Instruction mix of one kernel in a hipcc -S output: the prologue (up to the first s_barrier) and totals,
plus the register/LDS figures the assembler reports.  Usage: asm_report.py file.s [mangled-name-substring]"""
import re
import sys


def main(path, name="k_windowsILb1E"):
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"{name} not found")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    lines = [ln.strip() for ln in s[i:j].split("\n")]
    ins = [ln for ln in lines if ln and not ln.startswith((";", ".")) and not ln.endswith(":")]
    k = next((n for n, ln in enumerate(ins) if ln.startswith("s_barrier")), len(ins))

    def mix(seq):
        c = {}
        for ln in seq:
            op = ln.split()[0]
            key = ("buffer_load" if op.startswith("buffer_load") else "s_load" if op.startswith("s_load")
                   else "global_load" if op.startswith("global_load") else "ds_read" if op.startswith("ds_read")
                   else "ds_write" if op.startswith("ds_write") else "s_waitcnt" if op == "s_waitcnt"
                   else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else op)
            c[key] = c.get(key, 0) + 1
        return dict(sorted(c.items()))

    print(m.group(1))
    print("  prologue (to first s_barrier):", len(ins[:k]), mix(ins[:k]))
    print("  whole kernel:", len(ins), mix(ins))
    meta = s[j:j + 4000]
    for key in ("NumVgprs", "NumSgprs", "ScratchSize", "Occupancy", "LDSByteSize"):
        mm = re.search(r"; " + key + r":\s*(\S+)", s[i:j + 4000])
        if mm:
            print(f"  {key}: {mm.group(1)}")


if __name__ == "__main__":
    main(*sys.argv[1:])

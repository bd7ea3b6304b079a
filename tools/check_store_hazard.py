"""Scan gfx950 assembly (hipcc --save-temps) for a >8-byte vector-memory store whose data VGPRs
are overwritten by the very next VALU instruction (no wait states in between).  Such a pair
corrupted stored data in the persistent forward.  Usage:
  python tools/check_store_hazard.py file.s [...]"""
import re
import sys

STORE = re.compile(r"^\s*(buffer|global|flat)_store_dwordx([234])\s+(?:v\[\d+:\d+\],\s*)?v\[(\d+):(\d+)\]|"
                   r"^\s*buffer_store_dwordx([234])\s+v\[(\d+):(\d+)\]")
VDST = re.compile(r"^\s*v_\w+\s+v(?:\[(\d+):(\d+)\]|(\d+))")


def regs_of_store(line):
    m = re.match(r"^\s*buffer_store_dwordx[34]\s+v\[(\d+):(\d+)\]", line)
    if m:
        return int(m.group(1)), int(m.group(2))
    m = re.match(r"^\s*(?:global|flat)_store_dwordx[34]\s+v(?:\[\d+:\d+\]|\d+),\s*v\[(\d+):(\d+)\]", line)
    if m:
        return int(m.group(1)), int(m.group(2))
    return None


def main():
    bad = 0
    for path in sys.argv[1:]:
        lines = open(path).read().splitlines()
        func = "?"
        for i, ln in enumerate(lines):
            if re.match(r"^_Z\w+:", ln):
                func = ln[:-1]
            r = regs_of_store(ln)
            if not r:
                continue
            j = i + 1
            while j < len(lines) and (not lines[j].strip() or lines[j].strip().startswith((";", "."))):
                j += 1
            if j >= len(lines):
                continue
            m = VDST.match(lines[j])
            if m:
                lo, hi = (int(m.group(1)), int(m.group(2))) if m.group(1) else (int(m.group(3)), int(m.group(3)))
                if not (hi < r[0] or lo > r[1]):
                    bad += 1
                    print(f"{path}:{i + 1}: {func}\n    {ln.strip()}\n    {lines[j].strip()}")
    print(f"{bad} hazard pair(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())

"""Scan gfx950 assembly for a >8-byte vector-memory store whose data VGPRs are overwritten by the
very next VALU instruction (no wait states in between).  Such a pair corrupted stored data in the
persistent forward (toolchain finding (b)).

  python tools/check_store_hazard.py file.s [...]          hipcc --save-temps assembly
  python tools/check_store_hazard.py --lib libfa_hip.so    every gfx950 code object embedded in a
                                                           built library (llvm-objdump disassembly)
Exit status 1 if any pair is found."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
VDST = re.compile(r"^\s*v_\w+\s+v(?:\[(\d+):(\d+)\]|(\d+))")
FUNC = re.compile(r"^(?:[0-9a-f]+ <)?(_Z\w+)>?:")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def regs_of_store(line):
    m = re.match(r"^\s*buffer_store_dwordx[34]\s+v\[(\d+):(\d+)\]", line)
    if m:
        return int(m.group(1)), int(m.group(2))
    m = re.match(r"^\s*(?:global|flat)_store_dwordx[34]\s+v(?:\[\d+:\d+\]|\d+),\s*v\[(\d+):(\d+)\]", line)
    if m:
        return int(m.group(1)), int(m.group(2))
    return None


def scan_text(name, text, out=print):
    """Number of hazard pairs in one assembly / disassembly listing."""
    bad = 0
    lines = text.splitlines()
    func = "?"
    for i, ln in enumerate(lines):
        f = FUNC.match(ln)
        if f:
            func = f.group(1)
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
                out(f"{name}:{i + 1}: {func}\n    {ln.strip()}\n    {lines[j].strip()}")
    return bad


def disassemble_library(path, arch="gfx950"):
    """[(name, disassembly)] of every `arch` code object in the .hip_fatbin section of a linked
    library or object (the section holds one offload bundle per translation unit)."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(BUNDLE_MAGIC), data)]
        out = []
        for n, s0 in enumerate(starts):
            piece = data[s0:starts[n + 1] if n + 1 < len(starts) else len(data)]
            pb, co = os.path.join(td, f"b{n}"), os.path.join(td, f"c{n}.co")
            open(pb, "wb").write(piece)
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={pb}",
                                f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={arch}", co], check=True,
                                 capture_output=True, text=True).stdout
            out.append((f"{os.path.basename(path)}#{n}", dis))
        return out


def main(argv):
    bad = 0
    if argv and argv[0] == "--lib":
        for path in argv[1:]:
            objs = disassemble_library(path)
            if not objs:
                print(f"{path}: no gfx950 code object found")
                return 2
            for name, dis in objs:
                bad += scan_text(name, dis)
    else:
        for path in argv:
            bad += scan_text(path, open(path).read())
    print(f"{bad} hazard pair(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

"""CPU checks of the assembly hazard scanner (tools/check_store_hazard.py): a
>8-byte vector-memory store whose data VGPRs the very next VALU instruction overwrites."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "check_store_hazard.py")

HAZARD = """_Zkernel:
	buffer_store_dwordx4 v[2:5], v14, s[24:27], s19 offen
	v_ashrrev_i32_e32 v2, 2, v13
	s_endpgm
"""
CLEAN = """_Zkernel:
	buffer_store_dwordx4 v[2:5], v14, s[24:27], s19 offen
	; sched_barrier mask(0x00000000)
	s_nop 1
	v_ashrrev_i32_e32 v2, 2, v13
	global_store_dwordx2 v[6:7], v[0:1], off
	v_lshl_add_u64 v[0:1], s[0:1], 0, v[4:5]
	s_endpgm
"""


def _run(tmp_path, text):
    f = tmp_path / "k.s"
    f.write_text(text)
    return subprocess.run([sys.executable, TOOL, str(f)], capture_output=True, text=True)


def test_store_hazard_detected(tmp_path):
    r = _run(tmp_path, HAZARD)
    assert r.returncode == 1 and "1 hazard pair(s)" in r.stdout


def test_store_hazard_clean(tmp_path):
    # a wait state in between, and an 8-byte store (not affected) followed by a write of its data
    r = _run(tmp_path, CLEAN)
    assert r.returncode == 0 and "0 hazard pair(s)" in r.stdout


def test_shipped_library_has_no_store_hazard():
    """The scanner over every gfx950 code object of the built product library (one per .hip
    translation unit), not only synthetic text."""
    import glob
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_store_hazard as H
    lib = os.path.join(ROOT, "tf_flash_attention_amd", "libfa_hip.so")
    objs = H.disassemble_library(lib)
    csrc = os.path.join(ROOT, "tf_flash_attention_amd", "csrc")

    def has_kernels(p):  # the unit's own text or a shared kernel header it includes (*_impl.h)
        text = open(p).read()
        impl = [ln.split('"')[1] for ln in text.splitlines() if ln.startswith('#include "') and '_impl.h"' in ln]
        return "__global__" in text + "".join(open(os.path.join(csrc, f)).read() for f in impl)
    # translation units with kernels (fa_api.hip has none)
    n_tu = sum(has_kernels(p) for p in glob.glob(os.path.join(csrc, "*.hip")))
    assert len(objs) == n_tu
    assert sum(d.count("buffer_store") + d.count("global_store") for _, d in objs) > 100
    found = []
    assert sum(H.scan_text(n, d, out=found.append) for n, d in objs) == 0, found


def test_setup_py_builds_through_make():
    """setup.py (the reference's setup.py / pyproject counterpart) drives the same make build."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "setup.py", "--name"], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == "tf_flash_attention_amd"
    r = subprocess.run([sys.executable, "setup.py", "--dry-run", "build_ext"], cwd=root, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "BuildHip: make -C" in r.stdout and "tf_flash_attention_amd" in r.stdout

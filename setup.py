"""Packaging for the MI355X build: the counterpart of the reference's setup.py / pyproject.toml
(/root/reference/setup.py:26-78, which runs `make` on the CUDA op library through a custom
build_ext).  Here build_ext runs `make -C tf_flash_attention_amd` (hipcc, gfx950) for the C-ABI
library libfa_hip.so, and, when TensorFlow(-ROCm) is importable, tf_op/build_tf_op.sh for the TF op
library the reference's unchanged flash_attention.py loads (flash_attention.py:77-78).

  python setup.py build_ext --inplace     # the in-tree build (what __graft_entry__.build() does)
  python setup.py bdist_wheel             # a wheel carrying libfa_hip.so (plus the TF op library if built)

The GPU tests and bench load the in-tree library; nothing here is needed to run them.
"""
import os
import subprocess
import sys

from setuptools import Extension, setup
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = "tf_flash_attention_amd"


class HipLibrary(Extension):
    """A prebuilt-by-make shared library: no sources for setuptools to compile."""

    def __init__(self, name, make_target):
        super().__init__(name, sources=[])
        self.make_target = make_target


class BuildHip(build_ext):
    def get_ext_filename(self, fullname):
        ext = self.ext_map.get(fullname)
        if isinstance(ext, HipLibrary):
            return os.path.join(*fullname.split(".")) + ".so"
        return super().get_ext_filename(fullname)

    def build_extension(self, ext):
        if not isinstance(ext, HipLibrary):
            return super().build_extension(ext)
        jobs = str(min(16, os.cpu_count() or 4))
        cmd = ["make", "-C", os.path.join(ROOT, PKG), f"-j{jobs}", ext.make_target]
        if self.dry_run:
            print("BuildHip: " + " ".join(cmd))
            return
        self.spawn(cmd)
        built = os.path.join(ROOT, PKG, "libfa_hip.so")
        dest = self.get_ext_fullpath(ext.name)
        if os.path.abspath(dest) != built:  # not --inplace: copy into the build tree
            os.makedirs(os.path.dirname(dest), exist_ok=True)
            self.copy_file(built, dest)
        # the TF op library, when TensorFlow is here (build_tf_op.sh reports and skips otherwise)
        tf_script = os.path.join(ROOT, PKG, "tf_op", "build_tf_op.sh")
        if subprocess.run([sys.executable, "-c", "import tensorflow"], capture_output=True).returncode == 0:
            self.spawn(["bash", tf_script])


setup(
    name="tf_flash_attention_amd",
    version="0.2.0",
    description="MI355X (gfx950) fused flash attention behind the tf_flash_attention API",
    packages=[PKG],
    package_data={PKG: ["libfa_hip.so", "tf_op/*.so", "tf_op/*.cc", "tf_op/*.sh"]},
    ext_modules=[HipLibrary(f"{PKG}.libfa_hip", "all")],
    cmdclass={"build_ext": BuildHip},
    python_requires=">=3.8",
    install_requires=["numpy", "torch"],
)

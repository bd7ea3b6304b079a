#!/bin/bash
# Builds the TensorFlow-ROCm op library (fa_tf_ops.cc over libfa_hip.so) that the reference's
# unchanged flash_attention.py loads (flash_attention.py:77-78):
#   bash tf_flash_attention_amd/tf_op/build_tf_op.sh [<reference flash_attention package dir>]
# Output: <dir>/kernel/flash_attention.so (default: tf_flash_attention_amd/tf_op/flash_attention.so).
# Needs a TensorFlow-ROCm installation (headers + libtensorflow_framework); this image has none,
# so here the script only reports that and exits 0.
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
PKG="$(dirname "$HERE")"
ROOT="$(dirname "$PKG")"
OUT="${1:+$1/kernel/flash_attention.so}"
OUT="${OUT:-$HERE/flash_attention.so}"
if ! python3 -c "import tensorflow" >/dev/null 2>&1; then
  echo "build_tf_op: TensorFlow is not importable here; the TF op library was not built (libfa_hip.so is the product)"
  exit 0
fi
make -C "$PKG" -j"${MAX_JOBS:-8}" >/dev/null
CFLAGS=$(python3 -c 'import tensorflow as tf; print(" ".join(tf.sysconfig.get_compile_flags()))')
LFLAGS=$(python3 -c 'import tensorflow as tf; print(" ".join(tf.sysconfig.get_link_flags()))')
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -DTENSORFLOW_USE_ROCM=1 $CFLAGS \
    -I"$ROOT/include" "$HERE/fa_tf_ops.cc" -L"$PKG" -lfa_hip -Wl,-rpath,"$PKG" $LFLAGS -o "$OUT"
echo "build_tf_op: wrote $OUT"

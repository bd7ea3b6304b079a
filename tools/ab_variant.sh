#!/bin/bash
# Builds a variant of the product library for an in-process A/B (tools/lib_ab.py): copies the package
# sources to a scratch dir, applies a python patch script to them, builds, and leaves
# tools/ab_build/<name>.so.  Usage: tools/ab_variant.sh NAME PATCH.py   (PATCH.py gets the csrc dir)
set -e
name=$1; patch=$2
root=$(cd "$(dirname "$0")/.." && pwd)
w=/tmp/ab_$name
rm -rf $w && mkdir -p $w/pkg && cp -r $root/tf_flash_attention_amd/csrc $root/tf_flash_attention_amd/Makefile $w/pkg/ && cp -r $root/include $w/include
python3 $patch $w/pkg/csrc
make -C $w/pkg -j8 libfa_hip.so > $w/build.log 2>&1 || { tail -20 $w/build.log; exit 1; }
mkdir -p $root/tools/ab_build && cp $w/pkg/libfa_hip.so $root/tools/ab_build/$name.so
echo built tools/ab_build/$name.so

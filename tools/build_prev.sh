#!/bin/bash
# Build a library variant for same-box A/B runs (bench.py and the tests load it with MIM_LIB=<out>).
#   tools/build_prev.sh [REV [OUT [FILE...]]]
# FILEs (csrc file names) are taken from git revision REV, the others from the work tree; with no
# FILE every source comes from REV.  Defaults: REV = HEAD, OUT = variants/libmim_prev.so.
set -e
REV=${1:-HEAD}
OUT=${2:-variants/libmim_prev.so}
shift $(( $# > 2 ? 2 : $# ))
FILES=${*:-"knn.hip ransac.hip sift.hip api.cpp group.cpp mim_internal.h mim_debug.h"}
D=computervision_objectdetection_featurematching_amd
TMP=$D/csrc_variant
rm -rf $TMP && cp -r $D/csrc $TMP && mkdir -p "$(dirname "$OUT")"
for f in $FILES; do git show "$REV:$D/csrc/$f" > "$TMP/$f"; done
python3 - "$TMP" "$OUT" <<'PY'
import os, subprocess, sys, tempfile
sys.path.insert(0, '.')
from computervision_objectdetection_featurematching_amd import build as B
src, out = sys.argv[1], sys.argv[2]
od = tempfile.mkdtemp()
objs = []
for f in B.SOURCES:
    o = os.path.join(od, f + '.o')
    subprocess.check_call([B.HIPCC, *B.FLAGS, *B.SRC_FLAGS.get(f, []), '-c', f'{src}/{f}', '-o', o], stderr=subprocess.DEVNULL)
    objs.append(o)
subprocess.check_call([B.HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', out, *objs, '-L/opt/rocm/lib', '-lrccl', '-Wl,-rpath,/opt/rocm/lib'])
PY
rm -rf $TMP
echo "$OUT"

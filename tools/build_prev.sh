#!/bin/bash
# Build the library of a git revision (default HEAD) into variants/libmim_prev.so for same-box A/B runs
# (bench.py and the tests load it with MIM_LIB=variants/libmim_prev.so).
set -e
REV=${1:-HEAD}
D=computervision_objectdetection_featurematching_amd
rm -rf $D/csrc_prev && mkdir -p $D/csrc_prev variants /tmp/prevobj
for f in knn.hip ransac.hip sift.hip api.cpp mim_internal.h mim_debug.h; do
  git show $REV:$D/csrc/$f > $D/csrc_prev/$f 2>/dev/null || cp $D/csrc/$f $D/csrc_prev/$f
done
python3 - <<'PY'
import subprocess, sys
sys.path.insert(0, '.')
from computervision_objectdetection_featurematching_amd import build as B
src = 'computervision_objectdetection_featurematching_amd/csrc_prev'
objs = []
for f in B.SOURCES:
    o = f'/tmp/prevobj/{f}.o'
    subprocess.check_call([B.HIPCC, *B.FLAGS, *B.SRC_FLAGS.get(f, []), '-c', f'{src}/{f}', '-o', o], stderr=subprocess.DEVNULL)
    objs.append(o)
subprocess.check_call([B.HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', 'variants/libmim_prev.so', *objs])
PY
rm -rf $D/csrc_prev
echo variants/libmim_prev.so

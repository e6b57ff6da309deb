# build libmim variants with extra defines, in parallel:
#   VARIANTS="name:-DX=1 -DY=2;name2:..." -> lib/variants/libmim_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p computervision_objectdetection_featurematching_amd/lib/variants
IFS=';'
pids=""
for v in $VARIANTS; do
  name="${v%%:*}"; flags="${v#*:}"
  MIM_EXTRA_FLAGS="$flags" MIM_BUILD_DIR="/tmp/mimvar_$name" python -c "
import sys; sys.path.insert(0, '.')
from computervision_objectdetection_featurematching_amd import build as b
b.SO = 'computervision_objectdetection_featurematching_amd/lib/variants/libmim_$name.so'
b.build(force=True)" > /tmp/mimvar_$name.log 2>&1 &
  pids="$pids $!"
done
IFS=' '
for p in $pids; do wait $p; done

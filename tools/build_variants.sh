# build libmim variants with extra defines: VARIANTS="name:-DX=1 -DY=2;name2:..." -> lib/variants/libmim_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p computervision_objectdetection_featurematching_amd/lib/variants
IFS=';'
for v in $VARIANTS; do
  name="${v%%:*}"; flags="${v#*:}"
  MIM_EXTRA_FLAGS="$flags" python -c "
import sys, shutil; sys.path.insert(0, '.')
from computervision_objectdetection_featurematching_amd import build as b
b.SO = 'computervision_objectdetection_featurematching_amd/lib/variants/libmim_$name.so'
b.build(force=True)"
done

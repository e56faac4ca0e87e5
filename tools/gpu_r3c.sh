#!/bin/bash
# Round-3 second measurement batch: the cfg5 one-stream roofline profile,
# every config at its own size (tools/gpu_configs.sh), then an A/B of $LIBS.
#   LIBS="base: x:tools/bin/x/libzrt.so" bash tools/gpu_r3c.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r03c}
bash tools/gpu_roofline.sh $tag cfg5 || exit $?
bash tools/gpu_configs.sh $tag > /dev/null || exit $?
echo "configs done"
if [ -n "$LIBS" ]; then
  bash tools/gpu_ab_full.sh $tag > /dev/null || exit $?
  echo "ab done"
fi

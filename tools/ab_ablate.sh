#!/bin/bash
# Per-kernel records->pairs timings (tools/ablate.py) for the base library and variants.
# Usage (GPU box): tools/ab_ablate.sh name1 name2 ...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
echo "base: $(timeout -k 10 150 python $REPO/tools/ablate.py 2>&1 | tail -1)"
for v in "$@"; do
  echo "$v: $(KARMA_LIB=$REPO/karma_amd/variants/libkarma_$v.so timeout -k 10 150 python $REPO/tools/ablate.py 2>&1 | tail -1)"
done

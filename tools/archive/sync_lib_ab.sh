#!/bin/bash
# Alternating processes, one library build each (tools/sync_lib_ab.py): the
# directories named in $LIBS (default: tools/ab_lib_old, a previous build
# copied in by hand, and the current mpich-pip_amd/lib), 3 rounds.
set -e
LIBS=${LIBS:-"tools/ab_lib_old mpich-pip_amd/lib"}
for k in 1 2 3; do
  for l in $LIBS; do timeout -k 10 120 python3 tools/sync_lib_ab.py $l; done
done

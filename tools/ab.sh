#!/bin/bash
# Build the kbench harness from a git revision (default HEAD) into tools/kbench/kbench_ref, for A/B
# timing against the working tree's tools/kbench/kbench in the same GPU session.
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
D=$(mktemp -d)
git archive "$REV" bitcaskdb_amd/csrc include tools/kbench | tar -x -C "$D"
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-value -Wno-unused-result -Xarch_host -msse4.2 -I "$D/include" \
  -I "$D/bitcaskdb_amd/csrc" "$D/tools/kbench/kbench.hip" -o tools/kbench/kbench_ref
rm -rf "$D"

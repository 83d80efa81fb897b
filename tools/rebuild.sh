#!/bin/bash
# Rebuild libbcw.so and the kbench harness (host-side; cross-compiles gfx950).
set -e
cd "$(dirname "$0")/.."
python bitcaskdb_amd/build.py > /dev/null
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-value -Wno-unused-result -Xarch_host -msse4.2 -I include -I bitcaskdb_amd/csrc \
  tools/kbench/kbench.hip -o tools/kbench/kbench

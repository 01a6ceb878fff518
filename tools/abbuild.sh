#!/bin/bash
# Build an A/B variant of libacoss_hip.so with extra defines into tools/abl/libabl_<name>.so
#   bash tools/abbuild.sh <name> [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/../acoss-1_amd/csrc"
N=$1; shift
mkdir -p ../../tools/abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I../../include \
  -Wno-unused-function -Wno-unused-variable "$@" -o ../../tools/abl/libabl_$N.so *.hip *.cpp -lz

#!/bin/bash
# Build engine libraries whose mailbox groups have a different number of workgroups (kMailGroup), for an
# A/B of SYNC latency with tools/sync_probe (LD_LIBRARY_PATH=ctstraffic_amd/build/mgN tools/sync_probe ...).
#   usage: bash tools/mailbox_group_ab.sh 8 4
set -euo pipefail
cd "$(dirname "$0")/.."
for n in "$@"; do
  d=ctstraffic_amd/build/mg$n
  mkdir -p "$d"
  objs=()
  for f in ctstraffic_amd/csrc/*.hip ctstraffic_amd/csrc/*.cpp; do
    o=$d/$(basename "$f").o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -Iinclude \
      -Ictstraffic_amd/csrc -DCTS_MAIL_GROUP=$n -c "$f" -o "$o" &
    objs+=("$o")
  done
  wait
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -Wl,-Bsymbolic \
    -Wl,--version-script=ctstraffic_amd/csrc/exports.map -o "$d/libcts_engine.so" "${objs[@]}" -Wl,-soname,libcts_engine.so
  echo "built $d/libcts_engine.so"
done

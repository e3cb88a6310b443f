#!/bin/bash
# Timing-only: two builds of the library on one box, alternated (A B A B), each timed in its own process:
# c3 table through tools/ab.py (both arms the same handle settings) and one c4/8 table rank through
# tools/strip_timing.py.   bash tools/lib_ab.sh libdfamd_old.so [libdfamd.so]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
B=$1; A=${2:-libdfamd.so}
for lib in "$A" "$B" "$A" "$B"; do
  echo "== $lib c3 table"
  DFAMD_LIB=$ROOT/digital-filtering_amd/$lib timeout -k 10 120 python3 "$ROOT/tools/ab.py" --config c3 --mode table \
      --events 0 --rounds 5 || exit 1
done
for lib in "$A" "$B" "$A" "$B"; do
  echo "== $lib c4/8 table rank"
  DFAMD_LIB=$ROOT/digital-filtering_amd/$lib timeout -k 10 120 python3 "$ROOT/tools/strip_timing.py" --config c4 \
      --mode table --replicate 0 --ns 8 --calls 200 || exit 1
done

#!/bin/bash
# Timing-only: build a kernel variant (extra defines) next to libdfamd.so and run
# tools/ab.py once per library, so two compile-time variants can be compared on one box.
#   tools/variant_ab.sh NAME "-DDEFINE ..." [ab.py args]   (e.g. --mode table --tune-a zstage=0 --tune-b zstage=1)
# Separate processes: expect ~4% placement noise between the two libraries' numbers.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
V="$1"; VDEFS="$2"; shift 2
[ -f "$ROOT/digital-filtering_amd/libdfamd_$V.so" ] || make -C "$ROOT/digital-filtering_amd" variant V="$V" VDEFS="$VDEFS" >&2
echo "{\"lib\": \"libdfamd.so\", \"ab\": $(python3 "$ROOT/tools/ab.py" "$@")}"
echo "{\"lib\": \"libdfamd_$V.so\", \"ab\": $(DFAMD_LIB="$ROOT/digital-filtering_amd/libdfamd_$V.so" python3 "$ROOT/tools/ab.py" "$@")}"

#!/bin/bash
# Builds an experimental variant of libfnnue.so into exp/libfnnue_<name>.so
# (bench it with FNNUE_LIB=..., tools/exp_run.sh).  The shipped sources are
# never edited: the csrc tree is copied to build/exp_<name>/, the optional
# patch (git diff format, paths relative to the repo root) is applied there,
# extra -D flags (the tunables FT_UNIT_ITEMS, SEG_UNIT_PLIES, PLAN_WG,
# FT_DEPTH) go to every HIP source.
#   usage: tools/exp_build.sh <name> [file.patch] [-DFLAG ...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
patch=""
if [ $# -gt 0 ] && [ -f "$1" ]; then patch=$(cd "$(dirname "$1")" && pwd)/$(basename "$1"); shift; fi
W=$ROOT/build/exp_$name
rm -rf "$W"; mkdir -p "$W/fishnet_amd" "$ROOT/exp"
make -s -C "$ROOT/fishnet_amd/csrc" -j8 ARCH=gfx950 >/dev/null
# timestamps kept: make rebuilds only what the patch touches (and what includes it)
cp -a "$ROOT/fishnet_amd/csrc" "$W/fishnet_amd/csrc"
cp -a "$ROOT/include" "$W/include"
if [ -n "$patch" ]; then sleep 1; (cd "$W" && patch -p1 --quiet < "$patch"); fi
# -D flags change every object: make cannot see them, so nothing may be reused
# (until round 4 a flags-only build silently reused the main objects)
if [ $# -gt 0 ]; then rm -rf "$W/fishnet_amd/csrc/build" "$W/fishnet_amd/libfnnue.so"; fi
make -s -C "$W/fishnet_amd/csrc" -j8 ARCH=gfx950 HIPFLAGS="--offload-arch=gfx950 --offload-compress $*" >/dev/null
cp "$W/fishnet_amd/libfnnue.so" "$ROOT/exp/libfnnue_$name.so"
echo "exp/libfnnue_$name.so"

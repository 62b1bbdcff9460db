#!/bin/bash
# Builds lib/variants/librt_<name>.so from a git revision's sources (default HEAD), for in-process
# A/B against the working tree's build (scripts/perf_variants.py). Usage: build_base_variant.sh [rev] [name]
set -eu
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" ray-tracing-gpu-vulkan_amd/csrc ray-tracing-gpu-vulkan_amd/Makefile include | tar -x -C "$T"
mkdir -p "$T/ray-tracing-gpu-vulkan_amd/lib"
make -s -C "$T/ray-tracing-gpu-vulkan_amd" variant NAME="$NAME" VFLAGS="${VFLAGS:-}" > /dev/null 2>&1
mkdir -p "$ROOT/ray-tracing-gpu-vulkan_amd/lib/variants"
cp "$T/ray-tracing-gpu-vulkan_amd/lib/variants/librt_$NAME.so" "$ROOT/ray-tracing-gpu-vulkan_amd/lib/variants/"
rm -rf "$T"
echo "built lib/variants/librt_$NAME.so from $REV"

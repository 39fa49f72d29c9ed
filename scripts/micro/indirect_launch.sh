#!/bin/bash
# Build scripts/micro/indirect_launch.hip with the engine's flags and with the
# host-sanitizer flags (and each sanitizer alone), run each (GPU box).
set -u
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
A="--offload-arch=gfx950 -std=c++17"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all"
mkdir -p ../../gpurun_out/il
$H $A -O3 -o ../../gpurun_out/il/o3 indirect_launch.hip || exit 1
$H $A -O1 -g -fno-omit-frame-pointer $SAN -o ../../gpurun_out/il/san indirect_launch.hip || exit 1
$H $A -O1 -g -fno-omit-frame-pointer -Xarch_host -fsanitize=address -o ../../gpurun_out/il/asan indirect_launch.hip || exit 1
$H $A -O1 -g -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -o ../../gpurun_out/il/ubsan indirect_launch.hip || exit 1
$H $A -O1 -g $SAN -Xarch_host -fno-sanitize=function -o ../../gpurun_out/il/san_nofunc indirect_launch.hip || exit 1
$H $A -O1 -g -o ../../gpurun_out/il/o1 indirect_launch.hip || exit 1
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0
for b in o3 o1 asan ubsan san san_nofunc; do
  echo "== $b"
  timeout -k 5 60 ../../gpurun_out/il/$b
  echo "rc=$?"
done

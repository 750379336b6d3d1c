# Per-kernel VGPRs / scratch / occupancy of one HIP source (hipcc remarks), one line each.
# usage: bash tools/kernel_resources.sh <file.hip> [grep-pattern]
f=$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c -x hip "$f" -o /tmp/kr.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/^Function Name:/ {if (n) print n" | "v" | "s" | "o; n=$3; v=s=o=""} /^VGPRs:/ {v="vgpr "$2} /^ScratchSize/ {s="scratch "$3} /^Occupancy/ {o="occ "$3} END {print n" | "v" | "s" | "o}' |
  c++filt | grep -E "${2:-.}"

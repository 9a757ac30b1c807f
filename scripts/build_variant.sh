#!/bin/bash
# Build an experimental variant of libmmni.so with extra -D flags (kernel ablations), e.g.
#   bash scripts/build_variant.sh build/var_noatomic.so -DMMNI_ABL=1
# Load it with MMNI_LIB=<path>.  Not used by the product path.
set -e
out=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$(dirname "$out")" /tmp/mmni_var
objs=()
for f in "$R"/multimodal_neuroimage_amd/csrc/*.hip; do
  o=/tmp/mmni_var/$(basename "$f").$$.o
  extra=""; case "$(basename "$f")" in mlp.hip|blockops.hip|mha.hip) extra="-mllvm -amdgpu-mfma-vgpr-form";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -w $extra "$@" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$out" "${objs[@]}"
rm -f "${objs[@]}"
echo "built $out"

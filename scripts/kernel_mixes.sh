#!/bin/bash
# The bench kernels' own VALU issue peaks: static VALU
# opcode mixes of the product build (hipcc --save-temps of csrc/*.hip,
# scripts/valu_mix.py), weighted by the per-opcode issue costs measured on the
# GPU (scripts/micro/valu_peak.hip op_kernel<OP>, <valu_peak json>), at each
# kernel's clock and achieved rate from its PMC summary (<pmc dir>/<tag>_<leg>_pmc.json).
# Runs on the CPU (hipcc cross-compiles); the GPU inputs are files.
#   usage: scripts/kernel_mixes.sh <valu_peak json> <pmc dir> <tag> <out json>
set -e
peak=$1; pmc=$2; tag=$3; out=$4
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
for f in straight branch branch_demod macro dds; do
    (cd $tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --save-temps -c \
        -o $tmp/$f.o $OLDPWD/distributed_processor_amd/csrc/$f.hip 2>/dev/null)
done
mix() {   # asm file, kernel symbol substring, name
    python3 scripts/valu_mix.py $tmp/$1-hip-amdgcn-amd-amdhsa-gfx950.s "$2" --json $tmp/mix_$3.json > /dev/null
    echo $tmp/mix_$3.json
}
args=(
    $(mix straight '_ZN5dpemu15straight_kernelILi0ELi1EE' straight_rows_fb1)
    $(mix branch '_ZN5dpemu13branch_kernelILi11ELi8EE' branch_11_8)
    $(mix branch '_ZN5dpemu13branch_kernelILi14ELi8EE' branch_14_8)
    $(mix branch_demod '_ZN5dpemu13branch_kernelILi75ELi8EE' branch_75_8)
    $(mix macro '_ZN5dpemu19macro_staged_kernelILi2ELb1ELi8EE' macro_staged_2_addid)
    $(mix dds '_ZN5dpemu15dds_tile_kernelE' dds_tile)
)
python3 scripts/kernel_valu_peak.py $peak "${args[@]}" \
    --pmc "straight_kernelILi0ELi1=$pmc/${tag}_ramsey_pmc.json" \
    --pmc "branch_kernelILi11=$pmc/${tag}_active_reset_pmc.json" \
    --pmc "branch_kernelILi14=$pmc/${tag}_lut_pmc.json" \
    --pmc "branch_kernelILi75=$pmc/${tag}_demod_pmc.json" \
    --pmc "macro_staged_kernel=$pmc/${tag}_rb_pmc.json" \
    --pmc "dds_tile_kernel=$pmc/${tag}_dds_pmc.json" \
    --validation profiles/r05_valu_model_check.json --out $out
rm -rf $tmp

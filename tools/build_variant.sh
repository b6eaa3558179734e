# Build an A/B variant of libmsa_hip with extra compile flags (here, on the CPU):
#   bash tools/build_variant.sh NAME "-DQ_WGCU=2 ..."
# -> music-analyst-ai_amd/variants/libmsa_hip_NAME.so (travels to the GPU box;
# tools/ab_bench.sh NAME loads it through MSA_LIB)
set -eo pipefail
cd "$(dirname "$0")/../music-analyst-ai_amd"
make -s libmsa_hip.so
V=$1; shift
O=build/v_$V
mkdir -p $O variants
for f in msa_scan msa_k3 msa_post msa_sort msa_api msa_merge msa_wcs; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Wall -Wno-unused-function \
      -munsafe-fp-atomics "$@" -c csrc/$f.hip -o $O/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libmsa_hip_$V.so $O/*.o build/msa_gen.o build/msa_build_id.o
echo "variants/libmsa_hip_$V.so"

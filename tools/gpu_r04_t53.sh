# text.csv's gather (k_col_gather) with nontemporal fast-slot loads: configs[2] A/B
export TMPDIR=/tmp; mkdir -p gpurun_out/r04_t53
bash tools/ab_env.sh r04_t53/ab "nt:MSA_GATHER_NT=1" "base:X=1" "nt_b:MSA_GATHER_NT=1" "base_b:X=1" "nt_c:MSA_GATHER_NT=1" "base_c:X=1" "nt_d:MSA_GATHER_NT=1" "base_d:X=1" || exit 1
echo __done__

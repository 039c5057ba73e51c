# per-conv timing of k_micro_dw (tuning build: DQNX_MDW_SKIP masks convs out, DQNX_MDW_SPW<l> overrides)
set -u
mkdir -p gpurun_out/dwexp
export DQNX_LIB=${DQNX_LIB:-multimodal-drl-rmc_amd/dqn/_lib/libdqnx_stamps.so}
run() { # tag envs...
  tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --net hybrid --batch 256 --no-cpu-baseline --no-extras --steps 50 --warmup 5 > gpurun_out/dwexp/$tag.json 2> gpurun_out/dwexp/$tag.err || return 1
  python -c "import json;d=json.load(open('gpurun_out/dwexp/$tag.json'));print('$tag',round(d['ms_per_step']*1e3,1),[(k['kernel'],round(k['avg_us'],1)) for k in d['kernels'] if k['kernel'] in ('micro_dw','micro_fwd','micro_dx')])"
}
for spec in ${RUNS:-base:DQNX_MDW_SKIP=0 only0:DQNX_MDW_SKIP=6 only1:DQNX_MDW_SKIP=5 only2:DQNX_MDW_SKIP=3}; do
  tag=${spec%%:*}; envs=${spec#*:}
  run $tag ${envs//,/ } || exit 1
done

cd $GRAFT_REPO_ROOT
for v in base fix0 fixplain base fix0 fixplain; do
  if [ $v = base ]; then L=""; else L="KARMA_LIB=$PWD/karma_amd/variants/libkarma_$v.so"; fi
  env $L timeout -k 10 200 python bench.py --cpu-baseline off --no-e2e > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); k=d['kernels_ms_per_step']; print('$v', d['ms_per_step'], k['kmer_profile'], k.get('kmer_profile_exc'), k['graph_code_partition'])"
done

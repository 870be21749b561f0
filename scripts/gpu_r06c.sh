TAG=r06c FIRST="parity or batch or inflight or tuning or shadow or golden or multigpu" SPECS="-|qstate=0" bash scripts/gpu_ab.sh || exit 1
for v in "--scaling strong" "--scaling strong --batch 0"; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-pmc $v > gpurun_out/r06c/c4.log 2>&1 || exit 1
  tail -1 gpurun_out/r06c/c4.log | cut -c1-200
done
for t in "-" "qstate=0" "tlists=0" "qstate=0;tlists=0"; do
  VHX_BENCH_MGPU1=1 timeout -k 10 200 python3 bench.py --scaling strong --steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-pmc --tune "$t" > gpurun_out/r06c/c4m.log 2>&1 || exit 1
  echo "$t"; tail -1 gpurun_out/r06c/c4m.log | cut -c1-200
done
VHX_LIB=voxelhex_amd/_lib/libvhx_chain.so timeout -k 10 200 python3 scripts/chain_profile.py gpurun_out/r06c/chain

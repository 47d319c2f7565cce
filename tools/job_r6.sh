#!/bin/bash
# round-6 GPU job: parity of the current tree, then same-box A/B benches
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P=${JOB_PREFIX:-j}
run() {  # run <name> <secs> <cmd...>: stop the job on a crash-like exit
  local name=$1 secs=$2; shift 2
  local f="gpurun_out/${P}_$name.log" n=2   # a repeated step keeps every log
  while [ -e "$f" ]; do f="gpurun_out/${P}_${name}_r$n.log"; n=$((n + 1)); done
  timeout -k 10 "$secs" "$@" > "$f" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$f"
  if [ $rc -gt 1 ]; then echo "ABORT after $name"; exit $rc; fi
  return 0
}
summ() {
  for f in gpurun_out/${P}_bench*.log; do
    echo "$f"; tail -1 "$f" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['ms_per_launch'], {k:v['ms'] for k,v in d['kernels'].items() if v['ms']>0.4})" || true
  done
}
for s in "$@"; do
  case $s in
    parity) run parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread ;;
    graphs) run graphs 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -k "graph or rejects" ;;
    tests) run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    bench) run bench 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    benchfull) run benchfull 400 python bench.py ;;
    bv_*) v=${s#bv_}; run bench_$v 300 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    pv_*) v=${s#pv_}; run parity_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread ;;
    fv_*) v=${s#fv_}; run full_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread -k "v1 or determin or supercell"
          run family_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python -u -m pytest tests/test_gpu_family.py -x -q --timeout 400 --timeout-method thread ;;
    nve) run nve 900 python -u tools/nve_drift.py --cells 3 --steps 2000 --dt 1.0 --temp 600 ;;
    hfo2) run bench_hfo2 600 python bench.py --system hfo2 --steps 5 --warmup 1 --no-cpu-baseline ;;
    rankemu) run rankemu 900 python -u bench.py --rank-emulation 0,7 --steps 3 --warmup 1 ;;
    newtests) run newtests 900 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -k "bias_and_fcn or workspace or rejects" ;;
    nvetest) run nvetest 600 python -u -m pytest tests/test_gpu_native.py -x -q -s --timeout 400 --timeout-method thread -k nve_drift ;;
    gtrain) run gtrain 900 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    smoke_nl0) run smoke_nl0 300 env E3GNN_NL_BF16=0 python -c "import __graft_entry__ as g; g.smoke()" ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --profile-only --no-parity-check ;;
    pmcf) run pmcf 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    pmcw) run pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    pmcmops) run pmcmops 600 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_mops -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    proftraint) run proftraint 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_traint -o run -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    trainops) run trainops 300 python tools/prof_train_ops.py ;;
    opttests) run opttests 900 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread -k "bias_and_fcn or hfo2_resdat" ;;
    profbench) run profbench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_profbench -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fine-tune --no-parity-check ;;
    stamps_*) v=${s#stamps_}; run stamps_$v 300 python tools/stamps.py sevennet_finetuning_amd/variants/$v.so ;;
    tb) run tb 300 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    tb_noside) run tb_noside 300 env E3GNN_TRAIN_SIDE=0 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    tbs_*) v=${s#tbs_}; run tbs_$v 300 env E3GNN_TRAIN_SIDE=$v python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    tbsprof_*) v=${s#tbsprof_}; run tbsprof_$v 300 env E3GNN_TRAIN_SIDE=$v rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${P}_tbsprof_$v -o run -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    nvev_*) v=${s#nvev_}; run nvev_$v 900 python -u tools/nve_drift.py --cells 3 --steps 2000 --dt 1.0 --temp 600 --variant sevennet_finetuning_amd/variants/$v.so --label $v ;;
    fstamps_*) v=${s#fstamps_}; run fstamps_$v 300 python tools/stamps.py sevennet_finetuning_amd/variants/$v.so 23 fwd ;;
    summ) summ ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done

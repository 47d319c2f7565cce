#!/bin/bash
# GPU-box job: each GPU step under its own time limit; stop on any crash-like
# exit (fault/abort/segfault/timeout), continue only past ordinary test failures.
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    fullsize) step fullsize 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread ;;
    benchstrong) step benchstrong 600 python bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline ;;
    profstrong) step profstrong 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profstrong -o run --output-format csv -- python bench.py --strong --steps 2 --warmup 1 --profile-only --no-parity-check ;;
    testsall) step tests 900 python -m pytest tests -m gpu -q ;;
    layer) step layer 300 python -m pytest tests -m gpu -q -k layerwise ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 5 --warmup 2 ;;
    benchnl0) step benchnl0 600 env E3GNN_NODELIN=0 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benchnl) step benchnl 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benchq) step bench 600 python bench.py --steps 3 --warmup 1 --cpu-seconds 10 ;;
    benchf_*) step $s 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    benchf) step benchf 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    benchsync_*) step $s 600 env E3GNN_SYNC=1 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    benchmorton) step benchmorton 600 env E3GNN_BENCH_ORDER=morton python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    benchmorton_*) v=${s#benchmorton_}; step benchmorton_$v 600 env E3GNN_BENCH_ORDER=morton E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    t_*) t=${s#t_}; step t_$t 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k $t ;;
    bench10k) step bench10k 300 python bench.py --cells 11 --steps 5 --warmup 2 --no-cpu-baseline ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --profile-only --no-parity-check ;;
    proftrace) step proftrace 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/proftrace -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    bench2gloo) step bench2gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --same-device --no-cpu-baseline ;;
    traingraph) step traingraph 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "graph" ;;
    proftrain) step proftrain 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python bench_train.py --steps 10 --warmup 3 && mkdir -p gpurun_out/prof_train && cp /tmp/prof_train/*/*stats* /tmp/prof_train/*stats* gpurun_out/prof_train/ 2>/dev/null; ls gpurun_out/prof_train ;;
    traintests) step traintests 400 python -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread ;;
    benchtrain) step benchtrain 300 python bench_train.py --steps 10 --warmup 3 ;;
    benchtrain2_*) step $s 300 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrainsd) step benchtrainsd 300 env E3GNN_TRAIN_SI2_BLOCKS=0 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrainv_*) v=${s#benchtrainv_}; step benchtrain_$v 300 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrain2) step benchtrain2 300 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrainblk) step benchtrainblk 300 env E3GNN_TRAIN_DENSE_LINEAR=0 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrainlt) step benchtrainlt 300 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline --blas hipblaslt ;;
    benchtrainag) step benchtrainag 300 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline --autograd ;;
    proftrainx) step proftrainx 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trainx -o run --output-format csv -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    fullsize2) step fullsize2 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread -k edge_gradients ;;
    benchtraineager) step benchtraineager 300 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline --eager ;;
    benchd3) step benchd3 300 python bench_d3.py ;;
    profd3) step profd3 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_d3 -o run --output-format csv -- python bench_d3.py --no-cpu-baseline && mkdir -p gpurun_out/prof_d3 && cp /tmp/prof_d3/*/*stats* /tmp/prof_d3/*stats* gpurun_out/prof_d3/ 2>/dev/null; ls gpurun_out/prof_d3 ;;
    d3tests) step d3tests 300 python -m pytest tests/test_gpu_d3.py -x -q --timeout 200 --timeout-method thread ;;
    nativetests) step nativetests 300 python -m pytest tests/test_gpu_native.py -x -q -s --timeout 200 --timeout-method thread ;;
    md) step md 300 native/e3gnn_md sevennet_finetuning_amd/assets/sevennet0/weights.bin sevennet_finetuning_amd/assets/sevennet0/manifest.json 23 5 1.0 ;;
    mdpar) step mdpar 300 native/e3gnn_md_parallel sevennet_finetuning_amd/assets/sevennet0/weights.bin sevennet_finetuning_amd/assets/sevennet0/manifest.json 23 2 2 2 3 ;;
    prof10k) step prof10k 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10k -o run --output-format csv -- python bench.py --cells 11 --steps 3 --warmup 1 --profile-only ;;
    pmcf) step pmcf 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    pmcmops) step pmcmops 900 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_mops -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    pmcw) step pmcw 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    slp) step slp_build 600 env E3GNN_FUSED_FLAGS=" " python -c "import sevennet_finetuning_amd.build_lib as b; b.build(force=True)" && step benchslp 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    ptest) step ptest 600 python -m pytest tests/test_parallel.py -q ;;
    bench2) step bench2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --cells 11 --same-device --no-cpu-baseline ;;
    report) step report 300 python tools/parity_report.py ;;
    trainops) step trainops 300 python tools/prof_train_ops.py ;;
    pmctcp) step pmctcp 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum --kernel-trace --output-format csv -d gpurun_out/pmc_tcp -o run -- python bench.py --cells 11 --steps 1 --warmup 1 --profile-only ;;
    pmctcc) step pmctcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace --output-format csv -d gpurun_out/pmc_tcc -o run -- python bench.py --cells 11 --steps 1 --warmup 1 --profile-only ;;
    listc) step listc 120 rocprofv3 -L ;;
    pmcsq) step pmcsq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- python bench.py --cells 11 --steps 1 --warmup 1 --profile-only ;;
    pmcsq2) step pmcsq2 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/pmc_sq2 -o run -- python bench.py --cells 11 --steps 1 --warmup 1 --profile-only ;;
    pmcsqf) step pmcsqf 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_sqf -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    pmcsq2f) step pmcsq2f 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/pmc_sq2f -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    pmcsq3f) step pmcsq3f 600 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_sq3f -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    proftracev_*) v=${s#proftracev_}; step proftrace_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so rocprofv3 --kernel-trace --output-format csv -d gpurun_out/proftrace_$v -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    testsv_*) v=${s#testsv_}; step testsv_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread ;;
    benchv_*) v=${s#benchv_}; step bench_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    testsv_*) v=${s#testsv_}; step tests_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python -m pytest tests -m gpu -x -q ;;
    bench2self) step bench2self 600 python bench.py --gpus 2 --same-device --steps 2 --warmup 1 --cells 11 --no-cpu-baseline ;;
    paritydef) step paritydef 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread ;;
    stamps_*) v=${s#stamps_}; step stamps_$v 300 python tools/stamps.py sevennet_finetuning_amd/variants/$v.so ;;
    reportv_*) v=${s#reportv_}; step report_$v 300 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python tools/parity_report.py ;;
    benchtrain_notg) step benchtrain_notg 300 env E3GNN_TRAIN_TGEMM=0 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrain_nofl) step benchtrain_nofl 300 env E3GNN_TRAIN_FUSED_LOSS=0 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchtrain_none) step benchtrain_none 300 env E3GNN_TRAIN_FUSED_LOSS=0 E3GNN_TRAIN_TGEMM=0 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    btsplit_*) v=${s#btsplit_}; step btsplit_$v 300 env E3GNN_TG_SPLIT=${v//_/,} python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    btdense) step btdense 300 env E3GNN_TRAIN_IRREPS=0 python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    proftrainv_*) v=${s#proftrainv_}; step proftrain_$v 600 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_$v -o run --output-format csv -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    btcg_*) v=${s#btcg_}; step btcg_$v 300 env E3GNN_MLP_FWD_CG=$v python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    btmlp_*) v=${s#btmlp_}; cg=${v%_*}; wt=${v#*_}; step btmlp_$v 600 env E3GNN_MLP_FWD_CG=$cg E3GNN_MLP_W2T=$wt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp_$v -o run --output-format csv -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    proftracenl_*) v=${s#proftracenl_}; step proftracenl_$v 600 env E3GNN_NL_BF16=$v rocprofv3 --kernel-trace --output-format csv -d gpurun_out/proftracenl_$v -o run -- python bench.py --steps 1 --warmup 1 --profile-only --no-parity-check ;;
    benchnlm_*) v=${s#benchnlm_}; step benchnlm_$v 600 env E3GNN_NL_BF16=$v python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    fullv_*) v=${s#fullv_}; step full_$v 900 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread ;;
    tgb) step tgb 300 python tools/tgemm_bench.py --full ;;
    tgbs_*) v=${s#tgbs_}; step tgbs_$v 300 env E3GNN_TG_SMALL=$v python tools/tgemm_bench.py ;;
    btsmall_*) v=${s#btsmall_}; step btsmall_$v 300 env E3GNN_TG_SMALL=$v python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    btss_*) v=${s#btss_}; step btss_$v 300 env E3GNN_TG_SMALL_SPLIT=$v python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    tgbss_*) v=${s#tgbss_}; step tgbss_$v 300 env E3GNN_TG_SMALL_SPLIT=$v python tools/tgemm_bench.py ;;
    proftgb) step proftgb 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tgb -o run -- python tools/tgemm_bench.py --reps 3 --full ;;
    tgbv_*) v=${s#tgbv_}; step tgbv_$v 300 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python tools/tgemm_bench.py ;;
    btv_*) v=${s#btv_}; step btv_$v 300 env E3GNN_LIB=sevennet_finetuning_amd/variants/$v.so python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    btkarg_*) v=${s#btkarg_}; step btkarg_$v 300 env HIP_FORCE_DEV_KERNARG=$v python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    tgbkarg_*) v=${s#tgbkarg_}; step tgbkarg_$v 300 env HIP_FORCE_DEV_KERNARG=$v python tools/tgemm_bench.py ;;
    proftraint) step proftraint 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_traint -o run -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchdxc_*) v=${s#benchdxc_}; step benchdxc_$v 600 env E3GNN_DXC_SORTED=$v python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-check ;;
    btmlpbf_*) v=${s#btmlpbf_}; step btmlpbf_$v 300 env E3GNN_TRAIN_MLP_BF16=$v python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    gtrain) step gtrain 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread ;;
    benchmc_*) v=${s#benchmc_}; step benchmc_$v 600 python bench.py --model-config $v --steps 5 --warmup 2 --no-cpu-baseline ;;
    proftrain2) step proftrain2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train2 -o run --output-format csv -- python bench_train.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done

#!/bin/bash
# Every GPU check of a round, in one gpurun call.  Each phase named on the
# command line runs under its own time limit; the script stops at the first
# phase that faults, aborts or times out (gpurun rules: nothing more runs on
# the GPU after such a step).
#
#   /usr/local/graft/bin/gpurun -- 'bash tools/gpu_round.sh smoke tests bench'
#
# phases:
#   driver      what the driver runs at round end, in its words (pytest -x -q -m gpu, smoke(), bench.py)
#   smoke       __graft_entry__.smoke()
#   tests       the whole GPU suite (config-tagged parity tests first, tests/conftest.py)
#   tests_multi tests/test_gpu_multi.py only
#   bench       C2 bench line, 20 steps (the driver's N = 1 line); bench_c3, bench_c4: C3 / C4 on one GPU
#   rehearse    the multi-GPU modes on one GPU: one process 2-way split, 2 torchrun ranks under a
#               per-rank visibility mask, C4 over 8 one-process slots; rehearse8: 8 torchrun ranks on GPU 0
#   rehearse_fake  2 and 8 torchrun ranks on GPU 0 with the group joined through the stand-in RCCL
#   c5          C5 at size: the native (C++) system and the Python one
#   prof        rocprofv3 kernel traces of C2 (2 streams, 1 stream) and C3
#   prof_driver rocprofv3 kernel trace of the driver's exact bench command
#   pmc         PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) for C2 and C3, one counter group per run
#   parity      tools/parity_campaign.py, PARITY_CASES (3,000) random cases, seed PARITY_SEED (303)
#   lensweep    tools/len_sweep.py: GH/s and the three roofline fractions for every message length 0..130
#               (every layout a 10-digit search hits); lensweep_pmc: its SQ_INSTS_VALU pass
#   ab_padc     A/B of search_kernel_padc against the generic padding-block kernel (L = 45..53)
#   ab_padk     the same for search_kernel_padk<P, 1> (L = 109..117) and <P, 2> (L = 173..181)
#   ab_padk3    the same for <P, 3> (L = 237..245) and <P, 15> (L = 1005..1013), round 6
#   parity_pad  the padding-block parity tests and every kernel layout
#   ab          A/B of library variants: AB_LIBS="a.so b.so" (parity of each first, then alternating)
#   callsize    tools/call_size.py: GH/s of whole calls of 2^24 .. 2^34 nonces, one device and 8 slots on GPU 0
#   pmc_c2      the C2 PMC passes only (with each kernel's code hash in the summary, tools/pmc_summary.py)
#   rehearse_one  2 torchrun ranks on GPU 0 (--rehearse-one-gpu) with the C4 step and the one-process C4 block
# Logs and profiles land in gpurun_out/$TAG (TAG defaults to r06).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
  # 1 = test failures / a wrong answer: reported, the next phase still runs;
  # anything else (fault, abort, timeout, signal) ends the call here
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return $rc
}
PYTEST="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rs"
BENCH="python3 bench.py --no-cpu-baseline"
D=distributed_bitcoin_minter_amd
for phase in "$@"; do
  case $phase in
    driver)
      step driver_tests 1200 python -m pytest tests/ -x -q -m gpu
      step driver_smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
      step driver_bench 400 python bench.py ;;
    smoke) step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step gpu_tests 1200 $PYTEST tests -m gpu -v ;;
    tests_multi) step gpu_tests_multi 600 $PYTEST tests/test_gpu_multi.py -m gpu -v ;;
    tests_k) step gpu_tests_k 600 $PYTEST tests -m gpu -v -k "${TESTS_K}" ;;
    bench) step bench_C2 300 python -u bench.py --steps 20 --warmup 5 ;;
    bench_c3) step bench_C3 300 $BENCH --config C3 --steps 20 --warmup 5 ;;
    bench_c4) step bench_C4 300 $BENCH --config C4 --steps 2 --warmup 1 ;;
    rehearse)
      step rehearse2_oneproc 300 $BENCH --gpus 2 --steps 3 --warmup 2 --rehearse-one-gpu
      step rehearse2_mask 400 env HIP_VISIBLE_DEVICES=0 python -u -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2
      step rehearse8_C4 300 $BENCH --config C4 --gpus 8 --rehearse-one-gpu --steps 1 --warmup 1 ;;
    rehearse8)
      # the driver's N = 8 launch, all 8 ranks masked onto GPU 0 (RCCL refuses: rendezvous gather)
      step rehearse8_torchrun 400 env HIP_VISIBLE_DEVICES=0 python -u -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 2 --warmup 2 ;;
    rehearse_fake)
      # the driver's N = 2 / N = 8 launch shapes with the group JOINED: the
      # library linked against the stand-in RCCL (tests/fake_rccl/), every rank
      # on GPU 0 -- the joined-group path real RCCL refuses on one GPU
      step rehearse2_fakerccl 400 env HIP_VISIBLE_DEVICES=0 BTCMINER_LIB=$PWD/tests/fake_rccl/libbtcminer_fakerccl.so \
        python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
        bench.py --gpus 2 --steps 3 --warmup 2
      step rehearse8_fakerccl 400 env HIP_VISIBLE_DEVICES=0 BTCMINER_LIB=$PWD/tests/fake_rccl/libbtcminer_fakerccl.so \
        python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29520 \
        bench.py --gpus 8 --steps 2 --warmup 2 ;;
    c5)
      step c5_native 300 python -u tools/bench_c5_native.py
      step c5_python 300 python -u tools/bench_c5.py ;;
    c5_sizing)
      # round 6: one miner driving 8 device slots (GPU 0 eight times), fixed 2^32 jobs against
      # rate-sized ones, alternating twice; then 4 one-slot miners the same way
      for i in 1 2; do
        for t in 0 300; do
          step c5_8slot_t${t}_$i 300 python -u tools/bench_c5.py --miners 1 --slots 8 --target-ms $t
        done
      done
      for t in 0 300; do step c5_4miners_t$t 300 python -u tools/bench_c5.py --target-ms $t; done ;;
    prof)
      step prof_C2 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_C2" -o run --output-format csv -- $BENCH --steps 5 --warmup 2
      step prof_C2_1stream 300 env BTCMINER_STREAMS=1 rocprofv3 --kernel-trace --stats -d "$OUT/prof_C2_1stream" -o run \
        --output-format csv -- $BENCH --steps 5 --warmup 2
      step prof_C3 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_C3" -o run --output-format csv -- $BENCH --config C3 \
        --steps 5 --warmup 2 ;;
    prof_driver)
      # the driver's exact bench command under the kernel trace: the line's
      # roofline.kernel_ms and rocprof's average for that kernel, same run
      step prof_driver 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_driver" -o run --output-format csv \
        -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    pmc)
      for C in C2 C3; do
        step pmc_${C}_fetch 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_${C}_fetch" -o f --output-format csv \
          -- python3 tools/prof_one.py $C 2
        step pmc_${C}_write 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_${C}_write" -o w --output-format csv \
          -- python3 tools/prof_one.py $C 2
        step pmc_${C}_sq 90 env PROF_ONE_LAUNCHES="$OUT/pmc_${C}_launches.json" rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
          SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE \
          -d "$OUT/pmc_${C}_sq" -o s --output-format csv -- python3 tools/prof_one.py $C 2
      done ;;
    ab_nbv2_tight)
      # <4, 2>, <12, 2> (control), <13, 2>, <14, 2> at 7 waves (BM_NBV2_TIGHT=0 build) against the product's 6
      step ab_nbv2_tight 300 env AB_LO=1000000000000000 AB_MAXWIN=0 \
        AB_LIBS="t7=$D/libbtcminer_t7.so" python -u tools/ab_lens.py 52,60-62 5 2147483648 ;;
    callsize) step call_size 300 python -u tools/call_size.py --out "$OUT/call_size.json" ;;
    callsize_ab)
      # the submission pool (round 6) against the thread-per-call build, twice, alternating
      # ($D/libbtcminer_spawn.so: the library built from commit 95a42c3, before the pool;
      # profiles/r06/call_size_ab/ holds the result)
      for i in 1 2; do
        step call_size_pool_$i 300 python -u tools/call_size.py --max-bits 30 --out "$OUT/call_size_pool_$i.json"
        step call_size_spawn_$i 300 python -u tools/call_size.py --max-bits 30 --lib $D/libbtcminer_spawn.so \
          --out "$OUT/call_size_spawn_$i.json"
      done ;;
    pmc_c2)
      C=C2
      step pmc_${C}_fetch 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_${C}_fetch" -o f --output-format csv \
        -- python3 tools/prof_one.py $C 2
      step pmc_${C}_write 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_${C}_write" -o w --output-format csv \
        -- python3 tools/prof_one.py $C 2
      step pmc_${C}_sq 90 env PROF_ONE_LAUNCHES="$OUT/pmc_${C}_launches.json" rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
        SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE \
        -d "$OUT/pmc_${C}_sq" -o s --output-format csv -- python3 tools/prof_one.py $C 2
      step pmc_summary 60 python3 tools/pmc_summary.py "$OUT" "$OUT" C2 ;;
    rehearse_one)
      step rehearse2_c4_one 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 2 --warmup 2 --rehearse-one-gpu ;;
    rehearse8_one)
      # the driver's N = 8 launch shape, every rank and the one-process child's 8 slots on GPU 0
      step rehearse8_c4_one 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 8 --steps 2 --warmup 3 --rehearse-one-gpu ;;
    pmc_c3)
      C=C3
      step pmc_${C}_fetch 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_${C}_fetch" -o f --output-format csv \
        -- python3 tools/prof_one.py $C 2
      step pmc_${C}_write 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_${C}_write" -o w --output-format csv \
        -- python3 tools/prof_one.py $C 2
      step pmc_${C}_sq 90 env PROF_ONE_LAUNCHES="$OUT/pmc_${C}_launches.json" rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
        SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE \
        -d "$OUT/pmc_${C}_sq" -o s --output-format csv -- python3 tools/prof_one.py $C 2
      step pmc_summary_c3 60 python3 tools/pmc_summary.py "$OUT" "$OUT" C3 ;;
    parity) step parity_campaign 600 python -u tools/parity_campaign.py ${PARITY_CASES:-3000} ${PARITY_SEED:-303} ;;
    lensweep) step len_sweep 600 python -u tools/len_sweep.py --max-len 130 ;;
    lensweep_long)
      # round 6: the padding-block layouts after K = 1, 2, 3, 7, 15 prefix blocks (padk<P, K>)
      step len_sweep_long 300 python -u tools/len_sweep.py --lengths 109-117,173-181,237-245,493-501,1005-1013 ;;
    lensweep_pmc)
      # one search per length under SQ_INSTS_VALU (one stream, no tail split:
      # dispatch order = plan order); merge on the CPU with len_sweep.py --merge
      step len_sweep_pmcpass 300 env BTCMINER_STREAMS=1 BTCMINER_TAIL=0 rocprofv3 --pmc SQ_INSTS_VALU \
        -d "$OUT/pmc_lensweep" -o p --output-format csv -- python3 tools/len_sweep.py --pmc-pass --max-len 130 ;;
    ab_padc) step ab_padc 600 python -u tools/ab_padc.py ${AB_REPS:-5} ;;
    ab_padk)
      step ab_padk1 300 env AB_LENS=109-117 python -u tools/ab_padc.py ${AB_REPS:-5}
      step ab_padk2 300 env AB_LENS=173-181 python -u tools/ab_padc.py ${AB_REPS:-5} ;;
    ab_padk3)
      # round 6: search_kernel_padk<P, 3> (L = 237..245) and <P, 15> (L = 1005..1013) against the generic kernel
      step ab_padk3 300 env AB_LENS=237-245 python -u tools/ab_padc.py ${AB_REPS:-5}
      step ab_padk15 300 env AB_LENS=1005-1013 python -u tools/ab_padc.py ${AB_REPS:-5} ;;
    structure)
      # C2's 11 launches against one 10-digit range of the same size, live clock
      step structure 300 python -u tools/ab_structure.py 8
      step structure_1stream 300 env BTCMINER_STREAMS=1 python -u tools/ab_structure.py 8
      step structure_notail 300 env BTCMINER_TAIL=0 python -u tools/ab_structure.py 8 ;;
    parity_pad) step parity_pad 300 $PYTEST tests/test_gpu_parity.py -m gpu -k "padding_block or every_kernel_layout" -q ;;
    ab)
      for lib in $AB_LIBS; do
        n=$(basename "$lib" .so)
        BTCMINER_LIB=$PWD/$lib step "parity_$n" 300 $PYTEST tests/test_gpu_parity.py -q -x || { echo "parity $n failed"; exit 1; }
      done
      L="$D/libbtcminer.so $AB_LIBS"
      step ab 1200 env AB_REPS=${AB_REPS:-5} python -u tools/ab_bench.py $L $L $L $L ;;
    *) echo "unknown phase $phase"; exit 2 ;;
  esac
done
echo "done ($(date +%T))"

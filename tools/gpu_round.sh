#!/usr/bin/env bash
# One GPU-box session: parity tests -> bench -> rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; a crash-type exit (fault, abort, segfault,
# time limit) ends the script without starting further GPU work.
#   usage: tools/gpu_round.sh [tag] [steps...]   steps: tests bench bench2 bench200 prof pmc transient extra cfg profcfg ab recv smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-run}"; shift || true
STEPS="${*:-tests bench prof}"
ROOT="$(pwd)"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"

fatal() {  # exit codes that mean the GPU step crashed or hung
  case "$1" in 0|1|2|5) return 1 ;; *) return 0 ;; esac
}

run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 5 "$OUT/$name.log"
  if fatal "$rc"; then echo "FATAL rc=$rc in $name; stopping" | tee -a "$OUT/steps.log"; exit "$rc"; fi
  return 0
}

pmc_refresh() {  # FETCH_SIZE pass over the bench -> gpurun_out/$TAG/pmc_traffic.json and profiles/pmc_traffic.json
  cd /tmp && run pmc 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc" -o bench -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-extras
  cd "$ROOT"
  python3 tools/pmc_traffic.py $(find "$OUT/pmc" -name "*counter_collection.csv" | head -1) "$OUT/pmc_traffic.json" 1048576 \
    > "$OUT/pmc_traffic.log" 2>&1 && cp "$OUT/pmc_traffic.json" profiles/pmc_traffic.json
}

rocminfo 2>/dev/null | grep -m3 -E "Marketing Name|gfx950" > "$OUT/device.txt" || true
nproc > "$OUT/host_cpus.txt"; lscpu 2>/dev/null | grep -m1 "Model name" >> "$OUT/host_cpus.txt" || true

for s in $STEPS; do
  case "$s" in
    testsvar) run gpu_tests_var 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout=300 --timeout-method thread -k "var or packed or zipf or mixed or every_length or smoke" ;;
    testsbuild) run gpu_tests_build 600 python -u -m pytest tests/test_gpu_parity.py tests/test_loopback.py -m gpu -x -v -rf --timeout=300 --timeout-method thread -k "build or loopback or verify_drops or receive_bench" ;;
    testslib) for t in ${TEST_LIBS}; do
             WTP_LIB="$ROOT/a3-reliable-transport_amd/lib/ab/$t.so" run "gpu_tests_$t" 600 python -u -m pytest tests -m gpu -x -v -rf --timeout=300 --timeout-method thread -k "${TEST_K:-not loopback and not bench_}"
           done ;;
    abcrcns) for nn in ${AB_NS:-16384 65536 262144 1048576}; do
               run "abcrc_n$nn" 300 python tools/ab_lib.py --what crc --n $nn ${AB_LIBS}
             done ;;
    abcrcalt) run abcrcalt 300 python tools/ab_lib.py --what crcalt --n ${AB_N:-1048576} ${AB_LIBS} ;;
    abcrc2m) run abcrc2m 300 python tools/ab_lib.py --what crc --n 2097152 ${AB_LIBS} ;;
    c5sq)  for lib in ${SQ_LIBS:-product}; do
             if [ "$lib" = product ]; then LP="$ROOT/a3-reliable-transport_amd/lib/libwtp_crc32.so"; else LP="$ROOT/a3-reliable-transport_amd/lib/ab/$lib.so"; fi
             WTP_LIB="$LP" run "sq_$lib" 400 bash tools/prof_pieces.sh "$TAG/sq_$lib"
             cd /tmp
             WTP_LIB="$LP" run "fetch_$lib" 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/sq_$lib/fetch" -o c5 \
               -- python3 "$ROOT/tools/prof_pieces.py" 3
             cd "$ROOT"
           done
           python3 tools/sq_json.py "$OUT/c5_counters.json" $(for lib in ${SQ_LIBS:-product}; do echo "$lib=$OUT/sq_$lib"; done) > "$OUT/sq_json.log" 2>&1 || true ;;
    c5fetch) for lib in ${SQ_LIBS:-product}; do  # FETCH_SIZE of the C5 launch, one pass per library build
             if [ "$lib" = product ]; then LP="$ROOT/a3-reliable-transport_amd/lib/libwtp_crc32.so"; else LP="$ROOT/a3-reliable-transport_amd/lib/ab/$lib.so"; fi
             cd /tmp
             WTP_LIB="$LP" run "fetch_$lib" 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$lib" -o c5 \
               -- python3 "$ROOT/tools/prof_pieces.py" 5
             cd "$ROOT"
           done
           python3 tools/c5_fetch_summary.py "$OUT/c5_fetch.json" $(for lib in ${SQ_LIBS:-product}; do echo "$lib=$OUT/fetch_$lib"; done) > "$OUT/c5_fetch.log" 2>&1 || true ;;
    profwin) python3 tools/rocprof_window.py $(find "$OUT/prof" -name "*kernel_trace.csv" | head -1) "k_fixed_braid<6" 20 \
               "$OUT/rocprof_timed_window.json" $(python3 -c "import json,sys;print([json.loads(l) for l in open('$OUT/prof.log') if l.startswith('{')][-1]['warmup_run'])") > "$OUT/profwin.log" 2>&1 || true ;;
    tests) # a stale PMC record (the shipped k_fixed_braid<6> code differs from the one it measured)
           # is refreshed first, so the record test reads the current kernel's traffic
           if ! python3 -c "import sys; sys.path[:0]=['tools','.']; import bench; sys.exit(0 if bench.pmc_traffic(1<<20, 'a3-reliable-transport_amd/lib/libwtp_crc32.so')[0] else 1)"; then
             echo "PMC record stale: refreshing before the tests" | tee -a "$OUT/steps.log"
             pmc_refresh
           fi
           run gpu_tests 900 python -u -m pytest tests -m gpu -v -rf --timeout=300 --timeout-method thread ;;
    bench) run bench 400 python bench.py --steps 20 --warmup 5 ;;        # the driver's invocation
    bench2) run bench2 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench200) run bench200 400 python bench.py --no-cpu-baseline ;;
    c4shard) run c4shard 400 python bench.py --steps 20 --warmup 5 --packets-per-rank 2097152 --no-cpu-baseline ;;
    c4gather) run c4gather 400 python bench.py --steps 20 --warmup 5 --gather-n1 --packets-per-rank 2097152 --no-cpu-baseline ;;
    prof)  cd /tmp && run prof 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
           cd "$ROOT" ;;
    profnox) cd /tmp && run profnox 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/profnox" -o bench -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras
           cd "$ROOT" ;;
    pmcnew) pmc_refresh ;;
    pmccfg) # FETCH_SIZE and WRITE_SIZE of every configs-leg kernel, one config per process and pass
           cd /tmp
           for row in c2 c5_1.1 c5_1.0 verify build; do
             for ctr in FETCH_SIZE WRITE_SIZE; do
               run "pmc_${row}_${ctr}" 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmccfg/$row" -o "${row}_${ctr}" \
                 -- python3 "$ROOT/tools/pmc_configs.py" $row 20
             done
           done
           cd "$ROOT"
           python3 tools/pmc_configs.py --summarize "$OUT/pmc_configs.json" $(for row in c2 c5_1.1 c5_1.0 verify build; do echo "$row=$OUT/pmccfg/$row"; done) \
             > "$OUT/pmc_configs.log" 2>&1 || true ;;
    c4ab)  run c4ab 600 python -u tools/c4_leg_ab.py --rounds ${C4AB_ROUNDS:-8} --steps 20 --out "$OUT/c4_leg_ab.json" ;;
    rehearse) run rehearse 400 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 ;;
    newtests) run gpu_tests_new 600 python -u -m pytest tests -m gpu -v -rf --timeout=300 --timeout-method thread \
             -k "rehearse or captured_on_torch or piece_ranges or equal_work_c4_leg or pipelined_gather_one_rank" ;;
    gev)   for k in ${GEV:-1 2 4}; do
             run "c4gather_k$k" 300 python bench.py --steps 20 --warmup 5 --gather-n1 --packets-per-rank 2097152 --gather-every $k --no-cpu-baseline --no-probe
           done ;;
    transient) run transient 200 python -u tools/transient.py --out "$OUT/transient.json" ;;
    pmc)   cd /tmp && run pmc 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$OUT/pmc" -o bench -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-probe
           cd "$ROOT" ;;
    profcfg) cd /tmp && run profcfg 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/profcfg" -o cfg -- python3 "$ROOT/tools/bench_configs.py" --only "${CFG_ONLY:-c2,c5,verify}" --out "$OUT/profcfg_configs.json"
           cd "$ROOT" ;;
    extra) run extra 900 python tools/bench_configs.py --out "$OUT/configs.json" ;;
    cfg)   run cfg 600 python tools/bench_configs.py --only "${CFG_ONLY:-c5,verify}" --out "$OUT/configs.json" ;;
    recv)  for m in cpu gpu; do for b in 64 1024; do
             P=$((20000 + RANDOM % 20000))
             timeout -k 10 60 ./a3-reliable-transport_amd/bin/wReceiver --bench 3 -p $P --crc $m --batch $b \
               > "$OUT/recv_${m}_${b}.json" 2> "$OUT/recv_${m}_${b}.err" &
             RP=$!; sleep 0.5
             timeout -k 10 30 ./a3-reliable-transport_amd/bin/wBlast -h 127.0.0.1 -p $P --seconds 3 --batch 64 \
               --corrupt 100 > "$OUT/blast_${m}_${b}.json" 2>&1
             wait $RP; rc=$?
             echo "recv $m $b rc=$rc: $(cat "$OUT/recv_${m}_${b}.json")" | tee -a "$OUT/steps.log"
             if fatal "$rc"; then echo "FATAL rc=$rc in recv"; exit "$rc"; fi
           done; done ;;
    ab)    for lib in a3-reliable-transport_amd/lib/ab/*.so; do
             v=$(basename "$lib" .so)
             WTP_LIB="$ROOT/$lib" run "ab_$v" 300 python tools/bench_configs.py --only "${CFG_ONLY:-c5}" --out "$OUT/ab_$v.json"
           done ;;
    listavail) run listavail 120 rocprofv3 --list-avail ;;
    contig) run contig 300 python tools/contig_probe.py --out "$OUT/contig.json" ;;
    xover) run xover 200 ./tools/bin/verify_crossover 400 ;;
    tl)    run tl 200 python tools/tl_probe.py --out "$OUT/tl_phases.json"
           cd /tmp
           run tlpmc1 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum \
             TCP_UTCL1_STALL_MULTI_MISS_sum --output-format csv -d "$OUT/tlpmc1" -o tl -- python3 "$ROOT/tools/tl_probe.py"
           run tlpmc2 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum \
             TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
             --output-format csv -d "$OUT/tlpmc2" -o tl -- python3 "$ROOT/tools/tl_probe.py"
           cd "$ROOT"
           python3 tools/tl_summary.py "$OUT/tl_phases.json" "$OUT/tl_counters.json" $(find "$OUT/tlpmc1" "$OUT/tlpmc2" -name "*counter_collection.csv") > "$OUT/tl_summary.log" 2>&1 || true ;;
    recvsmall) for m in cpu gpu; do for b in ${RECV_BATCHES:-1 10 64}; do
             P=$((20000 + RANDOM % 20000))
             timeout -k 10 60 ./a3-reliable-transport_amd/bin/wReceiver --bench 3 -p $P --crc $m --batch $b \
               > "$OUT/recv_${m}_${b}.json" 2> "$OUT/recv_${m}_${b}.err" &
             RP=$!; sleep 0.5
             timeout -k 10 30 ./a3-reliable-transport_amd/bin/wBlast -h 127.0.0.1 -p $P --seconds 3 --batch ${BLAST_BATCH:-64} \
               --corrupt 100 > "$OUT/blast_${m}_${b}.json" 2>&1
             wait $RP; rc=$?
             echo "recv $m $b rc=$rc: $(cat "$OUT/recv_${m}_${b}.json")" | tee -a "$OUT/steps.log"
             if fatal "$rc"; then echo "FATAL rc=$rc in recv"; exit "$rc"; fi
           done; done ;;
    split) run split 300 python tools/split_probe.py ;;
    footprint) run footprint 300 python tools/footprint_probe.py ;;
    copyprobe) run copyprobe 120 ./tools/bin/copyprobe ;;
    ualprobe) run ualprobe 120 ./tools/bin/ualprobe ;;
    winprobe) run winprobe 120 ./tools/bin/winprobe ;;
    abbuild) run abbuild 300 python tools/ab_lib.py --what build ${AB_LIBS} ;;
    abcrc) run abcrc 300 python tools/ab_lib.py --what crc --n ${AB_N:-1048576} ${AB_LIBS} ;;
    abc5) run abc5 300 python tools/ab_lib.py --what c5 ${AB_LIBS:-a3-reliable-transport_amd/lib/libwtp_crc32.so} ;;
    abc5x) # both library orders, 1 M and 64 K payloads (AB_LIBS = two libraries)
           set -- ${AB_LIBS}
           for nn in 1048576 65536; do
             run "abc5_n${nn}_fwd" 300 python tools/ab_lib.py --what c5 --rounds 30 --n $nn $1 $2
             run "abc5_n${nn}_rev" 300 python tools/ab_lib.py --what c5 --rounds 30 --n $nn $2 $1
           done ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    kbalt) for al in 0 1; do  # braided kernel, its ablations and the probes: one buffer vs alternating buffers
             KB_ALT=$al KB_ONLY="${KB_VARS:-braid512_prod,braid512_skel,braid512_nolut,braid512_nofold,braid512_noprio,read_probe_g256x512,strided_nt_d2_g512}" \
               KB_SUSTAIN=all KB_REPS=${KB_REPS:-3} KB_NS=${KB_NS:-100} run "kbalt$al" 200 ./tools/bin/kbench ${KB_N:-1048576} 10
           done ;;
  esac
done
echo "done" | tee -a "$OUT/steps.log"

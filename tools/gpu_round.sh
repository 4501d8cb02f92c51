#!/bin/bash
# The one GPU-session driver (GPU box, repo root).  Runs the listed steps in order, each under its own time
# limit, and stops at the first failing step.  Outputs land in gpurun_out/TAG/; a summary is printed last.
#
# Usage: tools/gpu_round.sh TAG step...
#   tests            the GPU suite (pytest -m gpu)
#   smoke            __graft_entry__.smoke()
#   bench            the bench line without the slow legs (drop-in, CPU baseline off)
#   full             the default bench line exactly as the driver runs it
#   map              the mapping bench leg alone (config 4)
#   prof             rocprofv3 kernel trace + stats of the headline bench (tracking legs only)
#   pmc              FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run per counter) of the headline bench
#   mprof            rocprofv3 kernel trace + stats of the mapping bench (config 4)
#   mpmc             map step + FETCH_SIZE / WRITE_SIZE passes of the mapping bench (render kernels, config 4)
#   mpmcab           mpmc for the culled and the reference tile lists (--map-binning culled / reference)
#   sq[=REGEX]       SQ issue / wait / LDS counters of the render kernels (or the kernels REGEX names; two
#                    passes, <= 8 SQ counters each)
#   squnit           SQ + FETCH / WRITE passes and the kernel trace of the drop-in unit's single-image render_bwd
#   msq=REGEX        SQ + FETCH / WRITE passes of the mapping bench's kernels matching REGEX
#   unit             host / device split of the unchanged-caller unit (tools/raster_unit_profile.py, config 3)
#   stream           tools/micro/stream: STREAM copy / triad GB/s (the measured HBM peak)
#   lock             render_bwd row-list lockstep statistics (tools/lockstep_stats.py, configs 3 and 4)
#   wgtime           per-workgroup timelines of the render kernels (tools/wgtime.py; needs _diag/libgsr_wgtime.so)
#   phase            render_fwd / render_bwd phase shares (tools/phase.py; needs _diag/libgsr_phase.so)
#   ab=MODES=TAGS    interleaved A/B (two rounds) of tools/raster_bench.py stage times between libgsr.so and
#                    each splatam_amd/_diag/libgsr_<tag>.so (build_variant on the CPU first);
#                    MODES = mode:config[,mode:config...], TAGS = tag[,tag...]   e.g. ab=dual_lean:3,dual:4=ablw
#   abbench=TAGS     interleaved A/B of the bench line (tracking + mapping values, render stage times)
#   abprof=TAGS      interleaved A/B (two rounds) of rocprofv3 kernel-trace averages of the headline bench's
#                    tracking kernels between libgsr.so and each _diag/libgsr_<tag>.so
#   mabprof=TAGS     interleaved A/B (two rounds) of the mapping bench's rocprofv3 kernel averages and it/s
#   seqab=TAGS       interleaved A/B (two rounds) of the bench's sequence leg
#   abfisher=TAGS    interleaved A/B (two rounds) of the Fisher leg: poses/s and its kernels' rocprofv3 averages
#   configs          tests/test_gpu_configs.py with -s (per-config parity statistics in configs.log)
#   drv              the driver's bench command (--steps 20 --warmup 5) and 100/10, interleaved, two rounds
#   drift            per-launch render_track durations over 5 frames of 40 iterations (tools/drift.py)
#   clk              GRBM_COUNT / GRBM_GUI_ACTIVE per render_track launch over the drift run (clock per launch)
#   sqab=TAGS        SQ instruction counts (VALU / SALU / LDS per launch) of render_track (SQRX: another kernel
#                    regex) for libgsr.so and each _diag/libgsr_<tag>.so
#   abdropin=TAGS    interleaved A/B (two rounds) of the bench line with the drop-in legs (unchanged-caller tracking loop,
#                    raster unit, their render stage times)
#   abflag=FLAG:V1,V2[,...]  interleaved A/B (two rounds) of the light bench line over the values of one bench.py
#                    flag, e.g. abflag=--fuse-render:1,0
TAG=${1:-x}; shift
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
LIGHT="--cpu-baseline off --dropin off --fisher off --mapping off --configs off --unfused-leg off --stage-breakdown off --sequence off"
lib_of() { [ "$1" = base ] && echo "$ROOT/splatam_amd/libgsr.so" || echo "$ROOT/splatam_amd/_diag/libgsr_$1.so"; }
for s in "$@"; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
             > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; } ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
             || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; } ;;
    bench) timeout -k 10 300 python bench.py --dropin off --cpu-baseline off > "$OUT/bench.log" 2>&1 \
             || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; } ;;
    full) timeout -k 10 500 python bench.py > "$OUT/full.log" 2>&1 || { echo "full bench failed"; tail -30 "$OUT/full.log"; exit 1; } ;;
    map) timeout -k 10 300 python bench.py --workload mapping --cpu-baseline off > "$OUT/map.log" 2>&1 \
             || { echo "map failed"; tail -30 "$OUT/map.log"; exit 1; } ;;
    prof) ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
             --output-format csv -- python "$ROOT/bench.py" --steps 40 --warmup 20 $LIGHT > "$OUT/prof.log" 2>&1 ) \
             || { echo "prof failed"; tail -20 "$OUT/prof.log"; exit 1; } ;;
    pmc) for C in FETCH_SIZE WRITE_SIZE; do
           ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc $C \
               --kernel-include-regex 'render_|gauss_bwd|preprocess|duplicate|tile_colscan' -T -d "$OUT/pmc_$C" -o run \
               --output-format csv -- python "$ROOT/bench.py" --steps 20 --warmup 20 $LIGHT > "$OUT/pmc_$C.log" 2>&1 ) \
               || { echo "pmc $C failed"; tail -20 "$OUT/pmc_$C.log"; exit 1; }
         done ;;
    mprof) ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/mprof" -o run \
             --output-format csv -- python "$ROOT/bench.py" --workload mapping --cpu-baseline off --dropin off \
             > "$OUT/mprof.log" 2>&1 ) || { echo "mprof failed"; tail -20 "$OUT/mprof.log"; exit 1; } ;;
    mpmc) timeout -k 10 300 python bench.py --workload mapping --cpu-baseline off > "$OUT/map.log" 2>&1 \
             || { echo "map failed"; tail -30 "$OUT/map.log"; exit 1; }
         for C in FETCH_SIZE WRITE_SIZE; do
           ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $C \
               --kernel-include-regex 'render_|gauss_bwd' -T -d "$OUT/pmc_map_$C" -o run --output-format csv \
               -- python "$ROOT/bench.py" --workload mapping --steps 5 --warmup 5 --cpu-baseline off \
               > "$OUT/pmc_map_$C.log" 2>&1 ) || { echo "pmc map $C failed"; tail -20 "$OUT/pmc_map_$C.log"; exit 1; }
         done ;;
    mpmcab) for B in culled reference; do  # tile cull A/B of the mapping kernels: times + FETCH / WRITE bytes
           timeout -k 10 300 python bench.py --workload mapping --cpu-baseline off --map-binning $B \
               > "$OUT/map_$B.log" 2>&1 || { echo "map $B failed"; tail -30 "$OUT/map_$B.log"; exit 1; }
           for C in FETCH_SIZE WRITE_SIZE; do
             ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $C \
                 --kernel-include-regex 'render_|gauss_bwd' -T -d "$OUT/pmc_map_${B}_$C" -o run --output-format csv \
                 -- python "$ROOT/bench.py" --workload mapping --steps 5 --warmup 5 --cpu-baseline off --map-binning $B \
                 > "$OUT/pmc_map_${B}_$C.log" 2>&1 ) || { echo "pmc map $B $C failed"; tail -20 "$OUT/pmc_map_${B}_$C.log"; exit 1; }
           done
         done ;;
    squnit) # the drop-in unit's single-image render_bwd (tools/raster_bench.py --mode single, config 3): SQ issue /
            # wait / LDS counters, FETCH / WRITE bytes and the kernel trace, one rocprofv3 run each
        G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
        G2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
        i=0
        for G in "$G1" "$G2" FETCH_SIZE WRITE_SIZE; do
          i=$((i+1))
          ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc $G --kernel-include-regex 'render_bwd' -T \
              -d "$OUT/squnit$i" -o run --output-format csv -- python "$ROOT/tools/raster_bench.py" --mode single \
              --iters 40 --warmup 10 > "$OUT/squnit$i.log" 2>&1 ) || { echo "squnit pass $i failed"; tail -20 "$OUT/squnit$i.log"; exit 1; }
        done
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/squnit_trace" -o run \
            --output-format csv -- python "$ROOT/tools/raster_bench.py" --mode single --iters 40 --warmup 10 \
            > "$OUT/squnit_trace.log" 2>&1 ) || { echo "squnit trace failed"; tail -20 "$OUT/squnit_trace.log"; exit 1; } ;;
    msq=*) RX=${s#msq=}  # SQ issue / wait counters + FETCH / WRITE of the mapping bench's kernels that RX names
        G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
        G2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
        i=0
        for G in "$G1" "$G2" FETCH_SIZE WRITE_SIZE; do
          i=$((i+1))
          ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $G --kernel-include-regex "$RX" -T \
              -d "$OUT/msq$i" -o run --output-format csv -- python "$ROOT/bench.py" --workload mapping --steps 5 --warmup 5 \
              --cpu-baseline off > "$OUT/msq$i.log" 2>&1 ) || { echo "msq pass $i failed"; tail -20 "$OUT/msq$i.log"; exit 1; }
        done ;;
    sq|sq=*) RX='render_'; [ "$s" != sq ] && RX=${s#sq=}
        G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
        G2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
        i=0
        for G in "$G1" "$G2"; do
          i=$((i+1))
          ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc $G --kernel-include-regex "$RX" -T \
              -d "$OUT/sq$i" -o run --output-format csv -- python "$ROOT/bench.py" --steps 20 --warmup 20 $LIGHT \
              > "$OUT/sq$i.log" 2>&1 ) || { echo "sq pass $i failed"; tail -20 "$OUT/sq$i.log"; exit 1; }
        done ;;
    unit) timeout -k 10 300 python tools/raster_unit_profile.py --n 200 --out "$OUT/raster_unit_profile.txt" \
             > "$OUT/unit.log" 2>&1 || { echo "unit failed"; tail -20 "$OUT/unit.log"; exit 1; } ;;
    stream) timeout -k 10 120 tools/micro/stream > "$OUT/stream.json" 2>&1 || { echo "stream failed"; exit 1; } ;;
    lock) timeout -k 10 200 python tools/lockstep_stats.py 3 128 > "$OUT/lockstep3.txt" 2>&1 && \
          timeout -k 10 200 python tools/lockstep_stats.py 4 128 > "$OUT/lockstep4.txt" 2>&1 || { echo "lock failed"; exit 1; } ;;
    wgtime) GSR_LIB=$ROOT/splatam_amd/_diag/libgsr_wgtime.so timeout -k 10 200 python tools/wgtime.py --config 3 \
              --out "$OUT/wgtime.json" > "$OUT/wgtime.log" 2>&1 || { echo "wgtime failed"; tail -20 "$OUT/wgtime.log"; exit 1; } ;;
    phase) timeout -k 10 200 python tools/phase.py 3 10 > "$OUT/phase.json" 2>&1 || { echo "phase failed"; tail -20 "$OUT/phase.json"; exit 1; } ;;
    ab=*) spec=${s#ab=}; MODES=${spec%%=*}; TAGS=${spec#*=}
          for r in 1 2; do
            for t in base ${TAGS//,/ }; do
              for c in ${MODES//,/ }; do
                m=${c%%:*}; cf=${c##*:}; f="$OUT/ab_${t}_${m}_${cf}_$r.json"
                GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 120 python tools/raster_bench.py --iters 60 --mode $m --config $cf \
                    > "$f" 2>&1 || { echo "ab $t $c failed"; tail -5 "$f"; exit 1; }
                python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stages_us']; print('ab', sys.argv[2], sys.argv[3], 'round', sys.argv[4], 'preprocess', s['preprocess'], 'duplicate', s['duplicate'], 'render_fwd', s['render_fwd'], 'render_bwd', s['render_bwd'], 'gauss_bwd', s['gauss_bwd'], 'ms', round(d['ms_per_frame'], 4))" "$f" $t $c $r | tee -a "$OUT/ab.txt"
              done
            done
          done ;;
    abprof=*) TAGS=${s#abprof=}
         for r in 1 2; do
           L="base ${TAGS//,/ }"; [ $r = 2 ] && L="$(echo $L | tr ' ' '\n' | tac | tr '\n' ' ')"
           for t in $L; do
             d="$OUT/abprof_${t}_$r"
             ( cd /tmp && export TMPDIR=/tmp && GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 300 rocprofv3 --kernel-trace --stats \
                 -d "$d" -o run --output-format csv -- python "$ROOT/bench.py" --steps 40 --warmup 20 $LIGHT \
                 > "$d.log" 2>&1 ) || { echo "abprof $t failed"; tail -20 "$d.log"; exit 1; }
             python - "$d" $t $r <<'PY' | tee -a "$OUT/abprof.txt"
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
ks = {}
for row in csv.DictReader(open(f)):
    if int(row["Calls"]) >= 40:
        ks[row["Name"].split("(")[0].split("<")[0].split("::")[-1]] = float(row["AverageNs"]) / 1000
print("abprof", sys.argv[2], "round", sys.argv[3], " ".join(f"{k} {v:.2f}" for k, v in sorted(ks.items())))
PY
           done
         done ;;
    mabprof=*) TAGS=${s#mabprof=}  # interleaved A/B (two rounds) of the mapping bench's kernel averages
         for r in 1 2; do
           L="base ${TAGS//,/ }"; [ $r = 2 ] && L="$(echo $L | tr ' ' '\n' | tac | tr '\n' ' ')"
           for t in $L; do
             d="$OUT/mabprof_${t}_$r"
             ( cd /tmp && export TMPDIR=/tmp && GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 300 rocprofv3 --kernel-trace --stats \
                 -d "$d" -o run --output-format csv -- python "$ROOT/bench.py" --workload mapping --steps 120 --warmup 60 \
                 --cpu-baseline off > "$d.log" 2>&1 ) || { echo "mabprof $t failed"; tail -20 "$d.log"; exit 1; }
             python - "$d" $t $r <<'PY' | tee -a "$OUT/mabprof.txt"
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
ks = {}
for row in csv.DictReader(open(f)):
    if int(row["Calls"]) >= 100:
        ks[row["Name"].split("(")[0].split("<")[0].split("::")[-1]] = float(row["AverageNs"]) / 1000
d = json.loads([l for l in open(sys.argv[1] + ".log") if l.startswith("{")][-1])
print("mabprof", sys.argv[2], "round", sys.argv[3], "it/s", d["value"], " ".join(f"{k} {v:.2f}" for k, v in sorted(ks.items())))
PY
           done
         done ;;
    seqab=*) TAGS=${s#seqab=}  # interleaved A/B (two rounds) of the sequence leg (config 3 SLAM frames)
         for r in 1 2; do
           L="base ${TAGS//,/ }"; [ $r = 2 ] && L="$(echo $L | tr ' ' '\n' | tac | tr '\n' ' ')"
           for t in $L; do
             f="$OUT/seqab_${t}_$r.log"
             GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 300 python bench.py $LIGHT --sequence on > "$f" 2>&1 \
                 || { echo "seqab $t failed"; tail -20 "$f"; exit 1; }
             python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['sequence']; print('seqab', sys.argv[2], 'round', sys.argv[3], 'frames/s', d['value'], 'phases', d['phases_ms'], 'per_frame', d['per_frame']['value'])" "$f" $t $r | tee -a "$OUT/seqab.txt"
           done
         done ;;
    abfisher=*) TAGS=${s#abfisher=}
         for r in 1 2; do
           L="base ${TAGS//,/ }"; [ $r = 2 ] && L="$(echo $L | tr ' ' '\n' | tac | tr '\n' ' ')"
           for t in $L; do
             d="$OUT/abfisher_${t}_$r"
             ( cd /tmp && export TMPDIR=/tmp && GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 300 rocprofv3 --kernel-trace --stats \
                 -d "$d" -o run --output-format csv -- python "$ROOT/bench.py" --steps 20 --warmup 5 --cpu-baseline off \
                 --dropin off --mapping off --configs off --unfused-leg off > "$d.log" 2>&1 ) \
                 || { echo "abfisher $t failed"; tail -20 "$d.log"; exit 1; }
             python - "$d" $t $r <<'PY' | tee -a "$OUT/abfisher.txt"
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
ks = {r["Name"].split("(")[0].split("<")[0].split("::")[-1]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f))}
d = json.loads([l for l in open(sys.argv[1] + ".log") if l.startswith("{")][-1])
print("abfisher", sys.argv[2], "round", sys.argv[3], "poses/s", d["fisher"]["value"], " ".join(
    f"{k} {ks[k]:.2f}" for k in ("gauss_mpack_kernel", "render_bwd_fisher_kernel", "gauss_bwd_fisher_kernel") if k in ks))
PY
           done
         done ;;
    abbench=*) TAGS=${s#abbench=}
          for r in 1 2; do
            ORDER="base ${TAGS//,/ }"
            [ $r = 2 ] && ORDER=$(echo $ORDER | tr ' ' '\n' | tac | tr '\n' ' ')  # round 2 in reverse order
            for t in $ORDER; do
              f="$OUT/abbench_${t}_$r.log"
              GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 300 python bench.py --cpu-baseline off --dropin off --fisher off \
                  --configs off --unfused-leg off > "$f" 2>&1 || { echo "abbench $t failed"; tail -20 "$f"; exit 1; }
              python - "$f" $t $r <<'PY' | tee -a "$OUT/abbench.txt"
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("abbench", sys.argv[2], "round", sys.argv[3], "frames/s", b["value"], "render_bwd", b["roofline"]["avg_us"],
      "render_fwd", b["stages_us"]["render_fwd"], "mapping it/s", (b.get("mapping") or {}).get("value"))
PY
            done
          done ;;
    abdropin=*) TAGS=${s#abdropin=}
          for r in 1 2; do
            ORDER="base ${TAGS//,/ }"
            [ $r = 2 ] && ORDER=$(echo $ORDER | tr ' ' '\n' | tac | tr '\n' ' ')
            for t in $ORDER; do
              f="$OUT/abdropin_${t}_$r.log"
              GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -k 10 400 python bench.py --cpu-baseline off --fisher off --mapping off \
                  --configs off --unfused-leg off > "$f" 2>&1 || { echo "abdropin $t failed"; tail -20 "$f"; exit 1; }
              python - "$f" $t $r <<'PY' | tee -a "$OUT/abdropin.txt"
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = b["dropin"]
print("abdropin", sys.argv[2], "round", sys.argv[3], "frames/s", b["value"], "dropin", d["value"], "raster_unit",
      d["raster_unit"]["value"], "render_bwd", d["render_bwd"]["avg_us"], "stages", d["stages_us"])
PY
            done
          done ;;
    abflag=*) spec=${s#abflag=}; FL=${spec%%:*}; VALS=${spec#*:}
          for r in 1 2; do
            for v in ${VALS//,/ }; do
              f="$OUT/abflag_${FL//-/}_${v}_$r.log"
              timeout -k 10 300 python bench.py $LIGHT $FL $v > "$f" 2>&1 || { echo "abflag $FL $v failed"; tail -20 "$f"; exit 1; }
              python - "$f" "$FL $v" $r <<'PY' | tee -a "$OUT/abflag.txt"
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("abflag", sys.argv[2], "round", sys.argv[3], "frames/s", b["value"], "kernel", b["roofline"]["kernel"],
      "avg_us", b["roofline"]["avg_us"], "stages_us", b["stages_us"])
PY
            done
          done ;;
    configs) timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -s -v -m gpu --timeout 400 \
             --timeout-method thread > "$OUT/configs.log" 2>&1 || { echo "configs failed"; tail -40 "$OUT/configs.log"; exit 1; } ;;
    drv) for r in 1 2; do  # the driver's own bench command against the builder's 100/10 runs, interleaved
           for sw in "20 5" "100 10"; do
             set -- $sw; f="$OUT/drv_s$1_w$2_$r.log"
             timeout -k 10 300 python bench.py --gpus 1 --steps $1 --warmup $2 > "$f" 2>&1 \
               || { echo "drv $sw failed"; tail -20 "$f"; exit 1; }
             python - "$f" "$1/$2" $r <<'PY' | tee -a "$OUT/drv.txt"
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("drv steps/warmup", sys.argv[2], "round", sys.argv[3], "frames/s", b["value"], "kernel_us", b["roofline"]["avg_us"],
      "launches", b["roofline"].get("launches_timed"))
PY
           done
         done ;;
    drift) ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/drift" -o run \
             --output-format csv -- python "$ROOT/bench.py" --steps 200 --warmup 5 --settle-ms 0 $LIGHT > "$OUT/drift.log" 2>&1 ) \
             || { echo "drift failed"; tail -20 "$OUT/drift.log"; exit 1; }
           python tools/drift.py "$OUT/drift" --skip 25 | tee "$OUT/drift.txt" ;;
    clk) ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE \
             --kernel-include-regex render_track -T -d "$OUT/clk" -o run --output-format csv \
             -- python "$ROOT/bench.py" --steps 200 --warmup 5 --settle-ms 0 $LIGHT > "$OUT/clk.log" 2>&1 ) \
             || { echo "clk failed"; tail -20 "$OUT/clk.log"; exit 1; }
         python tools/drift.py "$OUT/clk" --skip 25 --counters | tee "$OUT/clk.txt" ;;
    sqlds=*) TAGS=${s#sqlds=}  # LDS bank-conflict census of the fused tracking render per library (duplicated phases)
         for t in base ${TAGS//,/ }; do
           d="$OUT/sqlds_$t"
           ( cd /tmp && export TMPDIR=/tmp && GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -s KILL 200 rocprofv3 --pmc \
               SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
               --kernel-include-regex "${SQRX:-render_track}" -T -d "$d" -o run --output-format csv \
               -- python "$ROOT/bench.py" --steps 20 --warmup 5 $LIGHT > "$d.log" 2>&1 ) \
               || { echo "sqlds $t failed"; tail -20 "$d.log"; exit 1; }
           python - "$d" $t <<'PY' | tee -a "$OUT/sqlds.txt"
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
n = max(len(v) for v in acc.values()) // 1
launches = len(set(r["Dispatch_Id"] for r in csv.DictReader(open(f))))
print("sqlds", sys.argv[2], "launches", launches, " ".join(f"{k} {sum(v) / max(launches, 1):.4g}" for k, v in sorted(acc.items())))
PY
         done ;;
    sqab=*) TAGS=${s#sqab=}  # SQ instruction counts of the fused tracking render per library (VALU census by variants)
         for t in base ${TAGS//,/ }; do
           d="$OUT/sqab_$t"
           ( cd /tmp && export TMPDIR=/tmp && GSR_LIB_AB=1 GSR_LIB=$(lib_of $t) timeout -s KILL 200 rocprofv3 --pmc \
               SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
               --kernel-include-regex "${SQRX:-render_track}" -T -d "$d" -o run --output-format csv \
               -- python "$ROOT/bench.py" --steps 20 --warmup 5 $LIGHT > "$d.log" 2>&1 ) \
               || { echo "sqab $t failed"; tail -20 "$d.log"; exit 1; }
           python - "$d" $t <<'PY' | tee -a "$OUT/sqab.txt"
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("sqab", sys.argv[2], " ".join(f"{k} {sum(v) / len(v) / 1e6:.3f}M" for k, v in sorted(acc.items())), "launches",
      len(acc.get("SQ_INSTS_VALU", [])))
PY
         done ;;
    *) echo "unknown step $s"; exit 1 ;;
  esac
  echo "step $s ok"
done
python - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
for f in glob.glob(f"{out}/prof/**/run_kernel_stats.csv", recursive=True)[:1]:
    for r in list(csv.DictReader(open(f)))[:8]:
        print(r["Name"].split("(")[0][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
for name in ("bench.log", "full.log", "map.log"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        ls = [l for l in open(p) if l.startswith("{")]
        if ls:
            b = json.loads(ls[-1])
            rf = b.get("roofline", {})
            print(name, "value", b["value"], b["unit"], "render_bwd", rf.get("avg_us"), "frac", rf.get("frac"),
                  "render_fwd", (b.get("stages_us") or {}).get("render_fwd"))
            if b.get("fisher"):
                fi = b["fisher"]
                print("  fisher", fi.get("value"), "dropin", fi.get("dropin"))
for name in ("lockstep3.txt", "lockstep4.txt", "stream.json", "smoke.log", "phase.json"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        print(open(p).read().strip()[-1500:])
t = os.path.join(out, "tests.log")
if os.path.exists(t):
    print(open(t).read().strip().split("\n")[-1])
PY

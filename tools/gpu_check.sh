#!/bin/bash
# One GPU-box pass: engine parity, run-driver parity, a short bench.
# Each step has its own time limit; a crash / fault / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    engine) run t_engine 500 python -u -m pytest tests/test_gpu_engine.py -v --timeout 150 --timeout-method thread ;;
    run)    run t_run 400 python -u -m pytest tests/test_gpu_run.py -v --timeout 120 --timeout-method thread ;;
    smoke)  run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 300 python -u bench.py --steps 200 --no-cpu-baseline ;;
    benchfull) run benchfull 400 python -u bench.py ;;
    tb)     run tb 500 python -u tools/sweep.py --variants 2 --bands 32,64,128 --tpl 1,3,4,5,6,8 --mw 1,2 --turns 120 ;;
    tb16k)  run tb16k 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 8,16,32 --tpl 1,3,4,5,6,8 --mw 1,2 --turns 960 ;;
    pmcsq)  run pmcsq 300 bash tools/pmc_sq.sh ;;
    pmcsq1) run pmcsq1 300 env TAG=_k1 BENCH_ARGS="--tpl 1" bash tools/pmc_sq.sh ;;
    strips) run strips 300 python -u tools/strip_emulate.py ;;
    stripsk) run stripsk 400 python -u tools/strip_emulate.py --halo 120 --tpl 4,6,8 ;;
    auto)   run auto 400 python -u tools/strip_emulate.py --halo 120 --full ;;
    auto16k) run auto16k 300 python -u tools/strip_emulate.py --size 16384 --n 2 --halo 120 --full --turns 4800 ;;
    strips8) run strips8 500 python -u tools/strip_emulate.py --n 8 --halo 120 --tpl 1,4,6,8 --band 16,24,32,48,64,96 ;;
    dist)   run t_dist 400 python -u -m pytest tests/test_gpu_distributed.py -v --timeout 300 --timeout-method thread ;;
    tbk)    run tbk 400 python -u tools/sweep.py --variants 2 --bands 96,137,192 --tpl 6,8 --mw 1 --turns 240 ;;
    tbq)    run tbq 500 python -u tools/sweep.py --variants 2 --bands 0,64,128,137,200,240,274,300,400 --tpl 6,8 --mw 1 --turns 120 ;;
    tbq16k) run tbq16k 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0,16,20,24,32,48 --tpl 4,6,8 --mw 1 --turns 960 ;;
    skew)   run skew 500 python -u tools/sweep.py --variants 2 --bands 96,137,192 --tpl 6,8 --mw 1 --mv 0,1,2,3,4 --turns 240 ;;
    skew16k) run skew16k 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 16,20,24,32 --tpl 6,8 --mw 1 --mv 0,1,2,3,4 --turns 960 ;;
    tb7)    run tb7 400 python -u -m pytest tests/test_gpu_engine.py -v -k temporal_blocking --timeout 150 --timeout-method thread ;;
    bench78) run bench_k7 300 python -u bench.py --tpl 7 --no-cpu-baseline && run bench_k8 300 python -u bench.py --tpl 8 --no-cpu-baseline && run bench_auto 300 python -u bench.py --no-cpu-baseline ;;
    strips78) run strips78 400 python -u tools/strip_emulate.py --n 2,4,8 --halo 128 --tpl 0,7,8 --rccl direct ;;
    calib)  run calib 300 bash tools/calib/run.sh ;;
    sweep)  run sweep 400 python -u tools/sweep.py --variants 2,4,5,6 --bands 16,32,64,128,256 ;;
    c2def)  run c2def 300 python -u bench.py --size 5120 --steps 1000 --warmup 40 --c3-size 0 --no-cpu-baseline ;;
    c2sweep) run c2sweep 500 python -u tools/sweep.py --size 5120 --variants 2 --bands 16,24,32,48,64 --tpl 4,8,12,16 --mw 1 --mv 7,9,12 --turns 960 ;;
    sq65)   run sq65 300 bash tools/pmc_sq.sh ;;
    prof)   run prof 1100 bash tools/profile_bench.sh ;;
    newr5)  run newr5 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_run.py -v --timeout 200 --timeout-method thread -k "pinned_shape or driver_command or harness or refuses_persistent" ;;
    calib5) run calib5 200 tools/calib/stencil_issue 4000 5 && (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/calib5_kt" -o run --output-format csv -- "$OLDPWD/tools/calib/stencil_issue" 4000 3 > "$OLDPWD/gpurun_out/calib5_kt.log" 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OLDPWD/gpurun_out/calib5_pmc" -o run --output-format csv -- "$OLDPWD/tools/calib/stencil_issue" 1000 1 > "$OLDPWD/gpurun_out/calib5_pmc.log" 2>&1); echo "calib5 prof rc=$?" ;;
    abwc)   for l in new wc0 new wc0; do lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd.so; [ $l = new ] || lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd_$l.so; run abwc_65_$l 200 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 65536 --turns 80 --rounds 3 --shapes 30:336:524:20,30:536:524:20 && run abwc_16_$l 200 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 3 --shapes 14:316:106:32 && run abwc_5_$l 200 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 5120 --turns 960 --rounds 3 --shapes 14:128:203:32; done ;;
    stripsw) run stripsw8 400 python -u tools/tile_sweep.py --size 65536 --height 8448 --turns 128 --rounds 3 --grid 30,14/524,516,512,506/16,32/4,8,12 && run stripsw4 400 python -u tools/tile_sweep.py --size 65536 --height 16640 --turns 128 --rounds 3 --grid 30,14/524,516,512/16,32/4,8,12 ;;
    c2sw)   run c2sw 300 python -u tools/tile_sweep.py --size 5120 --turns 960 --rounds 3 --shapes 14:128:203:32,14:128:103:32,14:128:3:32,14:128:403:32,14:128:503:32,14:128:404:32,10:160:203:32,10:160:403:32,10:160:503:32,10:160:103:32,10:160:3:32,10:160:204:32,10:160:404:32 ;;
    abwc2)  for l in new wc0 new wc0; do lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd.so; [ $l = new ] || lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd_$l.so; run abwc2_16_$l 200 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 3 --shapes 14:316:106:32,14:316:108:32,14:316:206:32,14:316:506:32,14:316:104:32,14:352:512:16 && run abwc2_s8_$l 200 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 65536 --height 8448 --turns 128 --rounds 3 --shapes 14:352:512:16,14:512:512:32,14:352:524:16,14:320:512:32 && run abwc2_s4_$l 200 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 65536 --height 16640 --turns 128 --rounds 3 --shapes 14:704:524:32,14:352:512:16,14:704:516:32 && run abwc2_s2_$l 300 env GOL_AMD_LIB=$lib python -u tools/tile_sweep.py --size 65536 --height 33024 --turns 64 --rounds 3 --shapes 30:336:524:20,30:536:524:20,14:704:524:32,14:720:524:24,30:336:524:16,14:352:512:16; done ;;
    stripsw4b) run stripsw4b 400 python -u tools/tile_sweep.py --size 65536 --height 16640 --turns 128 --rounds 3 --shapes 14:704:524:32,14:490:512:24,14:490:512:32,30:232:512:24,30:228:512:24,14:309:512:16,14:309:512:32,14:206:516:16,30:194:516:16,14:416:516:16,14:640:524:32,14:693:524:24,14:555:524:32,14:832:524:16,14:448:512:16,14:560:516:16 ;;
    wide65) run wide65 500 python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:20,30:344:524:20,62:472:532:20,62:448:532:32,62:344:524:20,62:456:532:24,62:472:132:20,62:608:540:16,62:600:540:20,30:536:524:20,14:720:524:24 ;;
    prewarm) run prewarm 300 python -u tools/prewarm_probe.py 0,10,30,60,100,300 && for i in 1 2 3; do run b20v$i 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1; run b20nv$i 200 env GOL_PIN_VERIFY_MS=0 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1; done ;;
    ord7)   run ord7t 300 python -u -m pytest tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -k "halo_wave or test_tile_code_pinned" && run ord7ab 400 python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:20,30:336:724:20,30:336:724:24,30:344:724:20,30:336:524:24,14:720:524:24 && run ord7ab2 400 python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:724:20,30:336:524:20,30:336:724:24,30:336:524:24 ;;
    retune16) run retune16 400 env GOL_AUTOTUNE=2 GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 16384 --auto --turns 640 --rounds 3 --shapes 14:316:106:32,14:320:108:32,14:316:206:32,14:320:112:32,14:352:512:16,14:316:506:32,30:320:512:32,30:320:112:32,30:320:516:32,30:352:516:16,14:448:108:32,14:456:112:24 ;;
    retune5) run retune5 300 env GOL_AUTOTUNE=2 GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3 --shapes 14:128:203:32,14:128:104:32,14:128:204:32,14:128:106:32,10:160:104:32,14:128:504:32,14:160:104:32 ;;
    bank)   run bank 200 tools/calib/vgpr_bank_probe 2000 ;;
    deep65) run deep65 500 python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:24,30:592:540:24,30:600:540:20,30:561:540:24,30:616:540:12,30:608:540:16,30:464:532:24,30:472:532:20,30:552:524:12,30:528:524:24,30:336:524:24 ;;
    ord8)   run ord8t 400 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u -m pytest tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -k "halo_wave or (test_tile_code_pinned and (824 or 812 or 806 or 524))" && run ord8ab 500 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:24,30:336:824:24,30:336:824:20,30:336:524:20,30:336:824:24 && run ord8s 500 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 65536 --height 8448 --turns 128 --rounds 3 --shapes 14:352:512:16,14:352:812:16,14:352:512:16,14:352:812:16 && run ord8s4 500 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 65536 --height 16640 --turns 128 --rounds 3 --shapes 14:704:524:32,14:704:824:32,14:704:524:32,14:704:824:32 && run ord8c3 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 3 --shapes 14:316:106:32,14:316:806:32,14:316:106:32,14:316:806:32 ;;
    iso)    run iso 300 tools/calib/turn_issue 3000 3 ;;
    ord9)   run ord9t 400 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u -m pytest tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -k "test_tile_code_pinned and (924 or 912 or 906)" && run ord9ab 500 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:24,30:336:924:24,30:336:824:24,30:336:524:24 ;;
    tvab)   for r in 1 2; do for V in 0 2 4 6; do run tvab_${V}_$r 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tv$V.so python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:24,30:336:824:24,30:336:924:24; done; done ;;
    pmc8)   for c in 524 824 924; do lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tv4.so; run pmc8_$c 400 env TAG=_$c GOL_AMD_LIB=$lib bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 24 --band 336 --tile 30,$c --turns 48; done ;;
    ord89)  run ord89t 500 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u -m pytest tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -k "halo_wave or (test_tile_code_pinned and (824 or 812 or 806 or 924 or 912 or 906))" ;;
    strip4c) run strip4c 500 python -u tools/tile_sweep.py --size 65536 --height 16640 --turns 144 --rounds 3 --shapes 14:704:524:32,30:336:524:24,30:320:524:24,30:330:524:24,30:347:524:24,14:720:524:24,14:694:524:32,30:336:524:20,14:704:524:32 && run strip2c 500 python -u tools/tile_sweep.py --size 65536 --height 33024 --turns 96 --rounds 3 --shapes 14:704:524:32,30:336:524:24,30:344:524:24,30:333:524:24,14:720:524:24,30:336:524:20,14:704:524:32 ;;
    ahead)  run iso2 300 tools/calib/turn_issue 3000 3 && for r in 1 2; do run ahead_t_$r 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:24,30:336:824:24 && run ahead_v_$r 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tv12.so python -u tools/tile_sweep.py --size 65536 --turns 120 --rounds 3 --shapes 30:336:524:24,30:336:824:24; done ;;
    th344)  for r in 1 2; do run th344_$r 400 python -u tools/tile_sweep.py --size 65536 --turns 240 --rounds 3 --shapes 30:336:524:24,30:344:524:20,30:336:524:20,30:340:524:20,30:344:524:20,30:336:524:24; done ;;
    svs)    run svs 300 python -u tools/single_vs_seq.py && (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/svs_kt" -o run --output-format csv -- python3 "$OLDPWD/tools/single_vs_seq.py" > "$OLDPWD/gpurun_out/svs_kt.log" 2>&1); echo "svs kt rc=$?" ;;
    vmode)  for i in 1 2 3; do run b20m0_$i 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 && run b20m1_$i 200 env GOL_PIN_VERIFY_MODE=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1; done ;;
    fullnx) run fullnx 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ;;
    full)   run full 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ;;
    stripx) run stripx 500 env GOL_AUTOTUNE_LOG=1 python -u tools/strip_emulate.py --n 2,4,8 --halo 128 --rccl direct --full --turns 768 ;;
    nobar)  run nobar 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 5120 --turns 960 --rounds 3 --shapes 30:64:8:32,30:64:308:32,30:64:4:32,30:64:304:32,10:160:4:32,10:160:304:32 && run nobar16 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/tile_sweep.py --size 16384 --turns 320 --rounds 3 --shapes 29:320:24:32,29:320:324:32 ;;
    sqc2)   run sqc2 300 env TAG=_c2 bash tools/pmc_sq.sh tools/kernel_run.py --size 5120 --mv 15 --tpl 32 --band 160 --tile 10,4 --turns 3200 && run sqc3 300 env TAG=_c3 bash tools/pmc_sq.sh tools/kernel_run.py --size 16384 --mv 15 --tpl 32 --band 320 --tile 29,124 --turns 640 ;;
    bench2g) run bench2g 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --c3-size 4096 --c3-turns 300 ;;
    bench20) run bench20 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    newt)   run newt 400 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "tile or small_board or rejects_tools or spin_timeout or snapshot_while or control_word or 5120 or random_vs_oracle" ;;
    c2tile) run c2tile 300 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --shapes 10:160:4:32,10:160:4:16,10:160:3:24,10:160:8:32,10:80:4:16,10:80:2:12,16:160:4:24,14:160:4:24,20:320:4:32,10:160:12:32,10:320:16:32,30:320:16:16,10:96:2:32,10:128:2:16,10:64:2:16,10:160:2:24,14:128:2:16,6:128:3:16,6:96:2:16 ;;
    autolog) run autolog 400 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 && run autolog16 400 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 16384 --auto --turns 960 && run autolog65 400 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 65536 --auto --turns 64 --rounds 2 ;;
    sqtile) run sqtile 300 bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 32 --band 576 --tile 30,40 --turns 128 && run sqskew 300 env TAG=_skew bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 7 --tpl 10 --band 137 --turns 100 ;;
    grid5)  run grid5 400 python -u tools/tile_sweep.py --size 5120 --turns 960 --rounds 2 --grid 10,14,8/2,3,4,6,8,106,108/16,24,32/8,12,16 ;;
    grid16) run grid16 400 python -u tools/tile_sweep.py --size 16384 --turns 320 --rounds 2 --grid 30,14,18/8,12,16,24,32,108,112,116,124,132/16,32/8,16 ;;
    grid65) run grid65 500 python -u tools/tile_sweep.py --size 65536 --turns 64 --rounds 2 --grid 30,14,62/16,24,32,40,116,124,132,140/16,32/8 ;;
    bigtile) run bigtile 300 python -u tools/tile_sweep.py --size 16384 --turns 320 --shapes 30:586:40:32,30:586:48:32,62:512:40:32,62:400:32:32,14:900:16:24,30:300:24:16 ;;
    bigtile65) run bigtile65 300 python -u tools/tile_sweep.py --size 65536 --turns 64 --rounds 2 --shapes 62:576:40:32,30:576:40:32,62:448:32:32,14:900:16:24,62:700:48:16 ;;
    tilesw5) run tilesw5 300 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --shapes 10:160:4:32,10:128:4:32,30:64:8:32,30:64:208:32,14:128:106:32,10:160:106:32,10:96:4:24 ;;
    tilesw16) run tilesw16 300 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 16384 --auto --turns 960 --shapes 29:320:24:32,29:320:124:32,29:320:224:32 ;;
    small65) run small65 400 python -u tools/tile_sweep.py --size 65536 --turns 96 --rounds 2 --shapes 30:576:140:32,14:320:106:32,14:352:106:16,14:336:106:24,14:352:206:16,14:224:104:16,14:352:6:16,10:256:104:32,10:288:104:16 && run small8448 400 python -u tools/tile_sweep.py --size 65536 --height 8448 --turns 192 --rounds 2 --shapes 62:192:132:32,14:320:106:32,14:352:106:16,14:336:106:24,14:352:206:16,14:224:104:16,14:352:6:16,10:288:104:16 ;;
    sqb) run sqc2b 300 env TAG=_c2b bash tools/pmc_sq.sh tools/kernel_run.py --size 5120 --mv 15 --tpl 32 --band 128 --tile 14,103 --turns 3200 && run sqc3b 300 env TAG=_c3b bash tools/pmc_sq.sh tools/kernel_run.py --size 16384 --mv 15 --tpl 32 --band 320 --tile 14,106 --turns 640 ;;
    kfix) run kfix 300 python -u tools/tile_sweep.py --size 5120 --turns 960 --rounds 2 --shapes 14:128:104:2,14:128:104:4,14:128:104:8,14:128:104:16,14:128:104:32,14:128:103:32,14:128:103:16 && run kfix16 300 python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 2 --shapes 14:320:106:2,14:320:106:4,14:320:106:8,14:320:106:16,14:320:106:32 ;;
    k20) run k20 400 python -u tools/tile_sweep.py --size 65536 --turns 80 --rounds 3 --shapes 14:960:116:20,14:960:16:20,14:984:16:20,14:960:216:20,30:600:140:20,30:600:40:20,14:448:8:20,14:448:108:20,14:960:16:32,30:576:140:32 ;;
    warm) for w in 5 60 5; do run warm$w 200 python -u bench.py --gpus 1 --steps 20 --warmup $w --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1; done; run warm40 200 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 ;;
    ovl8) run ovl8 400 python -u tools/strip_emulate.py --n 8,4 --halo 128 --rccl direct --turns 768 && run ovl8o 400 python -u tools/strip_emulate.py --n 8,4 --halo 128 --rccl direct --overlap --turns 768 ;;
    cold) run coldt 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "planner or interleaved or control_word or snapshot" && run coldb 300 env GOL_AUTOTUNE_LOG=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 && run coldb2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 ;;
    pin) for i in 1 2; do run pind$i 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 && run pin7_$i 300 env GOL_MULTI_VARIANT=7 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1; done ;;
    cold2) run coldt 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "planner or interleaved or control_word or snapshot" && for i in 1 2 3; do run coldb$i 300 env GOL_AUTOTUNE_LOG=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1; done ;;
    c2b) run c2b 300 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --shapes 14:128:104:32,14:122:104:32,14:128:103:32,14:122:103:32 && run c2bench 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --no-c1 ;;
    sweep16k) run sweep16k 300 python -u tools/sweep.py --size 16384 --turns 1000 --variants 1,2,4,5 --bands 8,12,16,24 ;;
  esac
done

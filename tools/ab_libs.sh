#!/bin/bash
# A/B of library builds on one GPU box (measurement aid, not product): each library in $LIBS
# (paths under nvidia-jetson-workload_amd/, default: the product library and
# lib/variants/libws_hip_base.so) runs the same short measurements, interleaved twice so box
# drift shows as a spread:
#   C2 RK4 (pinned to $C2PIN and autotuned), C3, C4, and the 8-rank C2 share (rank_timing,
#   stream-ordered / overlap at $XFER us per exchange).
# Each step has its own time limit; a failing step ends the script.
#   LIBS="lib/libws_hip.so lib/variants/libws_hip_base.so" tools/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS=${LIBS:-"lib/libws_hip.so lib/variants/libws_hip_base.so"}
C2PIN=${C2PIN:-dppy:2:-3:0}
XFER=${XFER:-0,40}
WHAT=${WHAT:-c2,c3,c4,slab8}
for round in 1 2; do
  for L in $LIBS; do
    echo "== round $round $L"
    export WS_HIP_LIB=nvidia-jetson-workload_amd/$L
    case ",$WHAT," in *,c2,*)
      timeout -k 10 150 python tools/pin_timing.py --config c2 --pins $C2PIN,auto --warmup 400 --steps 200 || exit 1;; esac
    case ",$WHAT," in *,c3,*)
      timeout -k 10 150 python tools/pin_timing.py --config c3 --pins auto --warmup 600 --steps 400 || exit 1;; esac
    case ",$WHAT," in *,c4,*)
      timeout -k 10 150 python tools/pin_timing.py --config c4 --pins auto --warmup 300 --steps 200 || exit 1;; esac
    case ",$WHAT," in *,c5,*)
      timeout -k 10 300 python tools/pin_timing.py --config c5 --pins auto --warmup 30 --steps 30 || exit 1;; esac
    case ",$WHAT," in *,slab8,*)
      timeout -k 10 200 python tools/rank_timing.py --config c2 --ranks 8 --xfer-us $XFER --variants off,on || exit 1;; esac
  done
done

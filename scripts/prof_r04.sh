#!/bin/bash
# Round-4 profiles on the GPU box (run from the repo root): for each config, a kernel trace +
# stats and one rocprofv3 --pmc pass per counter group over serialised frames
# (scripts/prof_pmc.sh), written under gpurun_out/prof_r04_<cfg>/.  Summarise here afterwards:
#   python scripts/traffic.py gpurun_out/prof_r04_<cfg> <cfg> --out profiles/r04 --skip 3
# usage: [TAG=r04f] scripts/prof_r04.sh [configs...]   (default: c3 c3b c5; TAG names the
# profile, default r04)
set -u
CFGS=${*:-"c3 c3b c5"}
for c in $CFGS; do
  frames=20
  [ "$c" = "c5" ] && frames=8
  scripts/prof_pmc.sh "${TAG:-r04}_$c" "$c" "$frames"
  rc=$?
  echo "prof $c rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

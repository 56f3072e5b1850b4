#!/bin/bash
# On the GPU box: runtime-length path timings over line / column block sizes (options GEN_TM, GEN_KN).
# usage: bash tools/gen_sweep.sh "TM KN" ...   (shapes: tools/time_generic.py defaults)
for cfg in "$@"; do
  set -- $cfg
  echo "== TM=$1 KN=$2"
  timeout -k 10 150 python tools/time_generic.py GEN_TM=$1 GEN_KN=$2 480,640,64 96,96,512 250,250,256 2048,2048,8 2>&1 | grep shape | cut -c1-75 || exit 1
done

#!/bin/bash
# On the GPU box: generic-path timings under the block-size options GEN_TM / GEN_KN.
for cfg in "2048 2048" "1024 2048" "2048 1024" "1024 1024" "512 1024"; do
  set -- $cfg
  echo "== KN=$1 TM=$2"
  timeout -k 10 120 python tools/time_generic.py GEN_KN=$1 GEN_TM=$2 2>&1 | grep shape | cut -c1-110 || exit 1
done

#!/bin/bash
# Staging-slot skew sweep for the fused 8-operand combine (tools/multi_gap_ab,
# HIP-event medians), interleaved over rounds: CHAIN8 fp16 at 128 MiB blocks
# and TREE8 fp32 at 32 MiB blocks.
for r in 1 2; do
  for sk in 0 2304 4352 8448 12544 33024 65792; do
    echo "## round $r skew $sk"
    timeout -k 10 120 tools/multi_gap_ab 128 10 $sk 16 | grep product || exit 1
    timeout -k 10 120 tools/multi_gap_ab 32 20 $sk | grep product || exit 1
  done
done

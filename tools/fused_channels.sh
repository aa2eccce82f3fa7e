#!/bin/bash
# tools/fused_channels under rocprofv3 --pmc, one pass per counter group
# (<= 4 TCC counters each), then the per-channel table:
#   per-channel passes  CH_RD_i / CH_WR_i = TCC_EA0_RDREQ / _WRREQ of TCC
#                       channel i (DIMENSION_INSTANCE), summed over the 8 XCDs
#   per-XCD passes      XCD_RD_k / XCD_WR_k, summed over the 16 channels
#   stall / level / size passes on the _sum counters
# The derived counters live in gpurun_out/fused_channels.yaml (written here,
# passed with -E).  Output: gpurun_out/fused_channels/<pass>/..., summary in
# gpurun_out/fused_channels.log (tools/fused_channels_summary.py).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fused_channels
mkdir -p $O
Y=$PWD/gpurun_out/fused_channels.yaml
python3 - > "$Y" <<'PY'
print("rocprofiler-sdk:\n  counters-schema-version: 1\n  counters:")
def ctr(name, expr, desc):
    print(f"  - name: {name}\n    description: '{desc}'\n    properties: []\n    definitions:\n"
          f"    - architectures:\n      - gfx950\n      expression: {expr}")
for i in range(16):
    for k, base in (("RD", "TCC_EA0_RDREQ"), ("WR", "TCC_EA0_WRREQ")):
        ctr(f"CH_{k}_{i:02d}", f"reduce(select({base},[DIMENSION_INSTANCE=[{i}]]),sum)", f"{base} of TCC channel {i}, all XCDs")
for x in range(8):
    for k, base in (("RD", "TCC_EA0_RDREQ"), ("WR", "TCC_EA0_WRREQ")):
        ctr(f"XCD_{k}_{x}", f"reduce(select({base},[DIMENSION_XCC=[{x}]]),sum)", f"{base} of XCD {x}, all channels")
PY
P=()
for i in 0 2 4 6 8 10 12 14; do
  j=$(printf %02d $((i + 1))); i2=$(printf %02d $i)
  P+=("ch$i2:CH_RD_$i2 CH_RD_$j CH_WR_$i2 CH_WR_$j")
done
for x in 0 2 4 6; do
  P+=("xcd$x:XCD_RD_$x XCD_RD_$((x + 1)) XCD_WR_$x XCD_WR_$((x + 1))")
done
P+=("stall:TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum")
P+=("level:TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum")
# write side of the EA (round 5): EA write-request stalls and DRAM write credit stalls
P+=("wstall:TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_sum")
P+=("dram:TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum")
# upstream of the EA: the CUs' side of the same requests
P+=("tcp:TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum")
P+=("tcpstall:TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum")
P+=("sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE")
P+=("tcc:TCC_BUSY_sum TCC_TAG_STALL_sum TCC_REQ_sum TCC_STREAMING_REQ_sum")
for e in "${P[@]}"; do
  name=${e%%:*}; ctrs=${e#*:}
  # PASSES="tcp sq" runs only the named passes
  if [ -n "$PASSES" ] && [[ " $PASSES " != *" $name "* ]]; then continue; fi
  echo "pass $name: $ctrs"
  timeout -s KILL 60 rocprofv3 -E "$Y" --pmc $ctrs --kernel-trace --output-format csv -d $O/$name -o run \
    -- tools/fused_channels ${ROUNDS:-12} > $O/$name.log 2>&1
done
python3 tools/fused_channels_summary.py $O > gpurun_out/fused_channels.log
cat gpurun_out/fused_channels.log

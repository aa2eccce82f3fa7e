#!/bin/bash
# Keep-alive variants against the idle-gap penalty (tools/idle_gap_probe.py):
# off, kernel no-op on its own queue, barrier packet on its own queue, kernel
# no-op on the calls' queue; period 40 us.
set -o pipefail
mkdir -p gpurun_out/ka
L=gpurun_out/ka/keepalive_ab.log
: > $L
run() {
  echo "== $1" >> $L
  env $2 timeout -k 10 120 python tools/idle_gap_probe.py --calls 150 2>&1 | grep "^gap" >> $L || exit 1
}
run off "MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=0"
run "default (barrier own 40)" "MPIR_CVAR_DUMMY=1"
run "kernel own 40" "MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=40 MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_KIND=kernel MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_QUEUE=own"
run "barrier own 40" "MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=40 MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_KIND=barrier MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_QUEUE=own"
run "kernel same 40" "MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=40 MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_KIND=kernel MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_QUEUE=same"

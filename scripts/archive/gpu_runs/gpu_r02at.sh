#!/bin/bash
# resolver backlog in the static order at 256 KiB: phases, and a 4-helper build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02at; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step ph_c5_8 200 env PBS_FUSED=1 PBS_DEBUG_PHASES=1 DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 8 vmimage 262144 1 || exit 1
C="PBS_FUSED=1,PBS_SCAN_DYN=1;PBS_FUSED=1,PBS_SCAN_DYN=0"
for lib in cur h4; do
  L=""; [ $lib = h4 ] && L=scripts/ab/libpbschunk_h4.so
  step ${lib}_c5_8 300 env DIAG_LIB=$L DIAG_CONFIGS="$C" python scripts/pass_diag.py 8 vmimage 262144 30 || exit 1
  step ${lib}_c5 300 env DIAG_LIB=$L DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 262144 5 || exit 1
  step ${lib}_c3 300 env DIAG_LIB=$L DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
done
echo done

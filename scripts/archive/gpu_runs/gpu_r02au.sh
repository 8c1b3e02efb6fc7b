#!/bin/bash
# six resolver helpers: config 5 static vs dynamic, headline static
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02au; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
C="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0"
for lib in cur h6; do
  L=""; [ $lib = h6 ] && L=scripts/ab/libpbschunk_h6.so
  step ${lib}_c5 300 env DIAG_LIB=$L DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 262144 5 || exit 1
  step ${lib}_c3 300 env DIAG_LIB=$L DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
  step ${lib}_a128 300 env DIAG_LIB=$L DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 131072 5 || exit 1
done
echo done

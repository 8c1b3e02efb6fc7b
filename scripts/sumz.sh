#!/bin/bash
# summary of a zstd A/B directory: corpus rates (compress ms), blob-stage lines, probe lines
d=${1:-.}
tail -1 $d/tests_zstd.log 2>/dev/null
for f in $d/rate_*; do echo "$(basename $f): $(python3 -c "
import json
out=[]
for l in open('$f'):
    l=l.strip()
    if l.startswith('{\"corpus'):
        d=json.loads(l); out.append(f\"{d['corpus']} {d['GiB/s']} ({d['ms']['compress_ms']})\")
print(', '.join(out))")"; done
for f in $d/blobs_*; do [ -f $f ] && echo "$(basename $f): $(grep -o '"blobs": {[^}]*}' $f | grep -o '"value": [0-9.]*, "ms": [0-9.]*, "kernel_ms": {[^}]*') $(grep -o '"verified": [a-z]*' $f | sort | uniq -c | tr '\n' ' ')"; done
[ -f $d/probe.log ] && grep "zstd probe" $d/probe.log | cut -c1-330

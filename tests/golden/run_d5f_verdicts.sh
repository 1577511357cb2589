#!/bin/bash
# Build container only: the reference's verdicts (20 s limit) on the faithful depth-5 sample,
# in 1,000-row chunks (one JSONL per chunk, so a cut-off run resumes at the next chunk).
cd "$(dirname "$0")"
PROCS=${PROCS:-6}
for start in $(seq ${FIRST:-0} 1000 10000); do
  out=ref/d5f_${start}_t20.jsonl
  [ -s "$out" ] && [ "$(wc -l < "$out")" -ge 1000 ] && continue
  python3 gen_reference_verdicts.py verdicts --input streams/force_free_d5_faithful.txt.gz \
    --out "$out" --start "$start" --stop $((start + 1000)) --timeout 20 --hard 90 --procs "$PROCS" || exit 1
done

#!/bin/bash
# Copy the summaries of one evidence session (gpurun_out/prof_TAG_*/summary.{txt,json}, written by
# tools/profile.sh / profile_cmd.sh) into profiles/ as PREFIX_<name>_summary.{txt,json}.
# Usage: tools/keep_profiles.sh TAG PREFIX      e.g. tools/keep_profiles.sh r04h r04
set -e
TAG=$1; PREFIX=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for d in "$ROOT"/gpurun_out/prof_"$TAG"_*; do
  [ -f "$d/summary.txt" ] || continue
  name=${d##*/prof_${TAG}_}
  cp "$d/summary.txt" "$ROOT/profiles/${PREFIX}_${name}_summary.txt"
  cp "$d/summary.json" "$ROOT/profiles/${PREFIX}_${name}_summary.json"
  for j in bench_trace.json out_trace.json; do
    [ -s "$d/$j" ] && cp "$d/$j" "$ROOT/profiles/${PREFIX}_${name}_run.json"
  done
  echo "$name"
done

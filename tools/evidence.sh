#!/bin/bash
# Roofline evidence for one workload on the GPU box (run from the repo root):
# kernel stats + PMC traffic (tools/profile_c2.sh), SQ VALU counts
# (tools/pmc_valu.sh), both summaries copied into profiles/ (so that the bench
# line below quotes them), then the bench line itself.
#   tools/evidence.sh TAG WORKLOAD [exact|closed] [bench args...]
#   -> profiles/r04_<wl>[c]_pmc_{traffic,valu}_TAG.json, gpurun_out/evidence_TAG/{<wl>.json, kernel_stats_<wl>.csv}
set -o pipefail
TAG=${1:?tag}; WL=${2:?workload}; FM=${3:-exact}; shift 3
lc=$(echo $WL | tr A-Z a-z); [ "$FM" = closed ] && lc=${lc}c
OUT=gpurun_out/evidence_$TAG
mkdir -p $OUT
tools/profile_c2.sh ${TAG}_$lc $WL $FM || exit 1
tools/pmc_valu.sh ${TAG}_$lc $WL $FM || exit 1
cp gpurun_out/prof_${TAG}_$lc/pmc_traffic.json profiles/r04_${lc}_pmc_traffic_$TAG.json
cp gpurun_out/valu_${TAG}_$lc/pmc_valu.json profiles/r04_${lc}_pmc_valu_$TAG.json
cp gpurun_out/prof_${TAG}_$lc/kernel_stats.csv $OUT/kernel_stats_$lc.csv
cp gpurun_out/valu_${TAG}_$lc/summary.txt $OUT/pmc_valu_summary_$lc.txt
timeout -k 10 400 python3 bench.py --workload $WL --fit-mode $FM "$@" > $OUT/$lc.json 2> $OUT/$lc.err || { tail -5 $OUT/$lc.err; exit 1; }
echo "evidence $WL $FM done"

# round-5 evidence at the final build: rocprofv3 kernel tables + PMC passes + bench lines (C3, C4),
# then the C3 rank-of-8 rehearsal
bash tools/gpu_evidence.sh r05k c3 "--steps 32" "--steps 64" && bash tools/gpu_evidence.sh r05k c4 "--steps 32" "--steps 32" || exit 1

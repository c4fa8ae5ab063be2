# Trace-ahead inside overlapped halves: parity, then C3 whole frame / one rank of 8 / C5 A/Bs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_quick.sh r06k "overlap or pixel_parts or gpu_parity" 1 || exit 1
bash tools/ab_env.sh r06k_c3 MPT_OVERLAP "-1 1 -1 1" --steps 32 || exit 1
MPT_OVERLAP=1 bash tools/ab_env.sh r06k_c3o MPT_OVERLAP_AHEAD "0 1" --steps 32 || exit 1
bash tools/ab_env.sh r06k_r8 MPT_OVERLAP_AHEAD "0 1 0 1" --emulate-rank-of 8 --steps 20 || exit 1
bash tools/ab_env.sh r06k_c5 MPT_OVERLAP_AHEAD "0 1" --workload c5 --steps 8 || exit 1

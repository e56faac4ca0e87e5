cd "${GRAFT_REPO_ROOT:-/root/repo}"
ZRT_WF_DEBUG=1 timeout -k 10 120 python -u tools/kbench.py --config cfg3 --spp 16 --reps 1 2>&1 | grep -v zrt_launch | head -20
for b in 1024 768 512; do ZRT_PARK_BLOCK=$b ZRT_WF_DEBUG=1 ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 120 python -u tools/kbench.py --config cfg3 --spp 64 --reps 2 2>&1 | grep -E "zrt_grid|mrays" | sort -u; done

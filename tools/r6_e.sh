set -u
cd "${GRAFT_REPO_ROOT}"
TESTS=0 NS=0 bash tools/r6_ab.sh r06_e "default tools/bin/ab/libjds_k6w4.so tools/bin/ab/libjds_k6np.so tools/bin/ab/libjds_k6w4np.so tools/bin/ab/libjds_r5inv.so" || exit 1
bash tools/r6_pmc.sh r06_e_pmc --steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-entropy --no-host-path || exit 1
echo all-done

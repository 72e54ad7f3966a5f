# A/B of prebuilt variants of hhfm_amd/lib (diagnostic): ab_libs.sh dir1 dir2 ...
cd "${GRAFT_REPO_ROOT:-.}"
export MB_ONLY=${MB_ONLY:-k2}
for d in "$@"; do
  cp $d/*.so hhfm_amd/lib/ && echo "== $d" && timeout -k 10 120 python scripts/microbench.py 2>/dev/null | grep -A1 '"c' | grep -v "^--" || exit 1
done

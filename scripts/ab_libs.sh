# A/B of prebuilt variants of hhfm_amd/lib (diagnostic): ab_libs.sh dir1 dir2 ...
# (variants from scripts/build_variants.sh; MB_ONLY selects the microbench legs)
cd "${GRAFT_REPO_ROOT:-.}"
export MB_ONLY=${MB_ONLY:-k2}
for d in "$@"; do
  cp $d/*.so hhfm_amd/lib/ && echo "== $d" && timeout -k 10 120 python scripts/microbench.py 2>/dev/null | python -c "
import json, sys
d = json.load(sys.stdin)
print({k: round(v['median_ms'], 3) for k, v in d.items() if isinstance(v, dict) and 'median_ms' in v})" || exit 1
done

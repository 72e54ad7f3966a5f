# A/B of prebuilt variants (scripts/build_variants.sh) on the DeepFM phase timer
# (AB_SCRIPT=scripts/afm_phases.py: the AFM one; its whole JSON is printed).
cd "${GRAFT_REPO_ROOT:-.}"
for d in "$@"; do
  if [ -n "$AB_SCRIPT" ]; then
    cp $d/*.so hhfm_amd/lib/ && echo "== $d" && timeout -k 10 200 python $AB_SCRIPT 2>/dev/null || exit 1
    continue
  fi
  cp $d/*.so hhfm_amd/lib/ && echo "== $d" && timeout -k 10 200 python scripts/dfm_phases.py 2>/dev/null | python -c "
import json, sys
d = json.load(sys.stdin)
print({k: v for k, v in d.items() if 'L1' in k or 'L3' in k})" || exit 1
done

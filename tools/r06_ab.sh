#!/bin/bash
# GPU box: round-6 A/B runs of generated-flash builds (tools/ab_flash.py),
# libraries from tools/diag_libs/ab_*.so.  Usage: tools/r06_ab.sh OUT "case;case;..."
# where case = "label|LIBS|ENV..." (ENV: SHAPE=..., CAUSAL=..., DTYPE=...).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
IFS=';' read -ra CASES <<< "$1"
for c in "${CASES[@]}"; do
  IFS='|' read -r label libs envs <<< "$c"
  echo "== $label" >&2
  env LIBS="$libs" ROUNDS=${ROUNDS:-8} $envs timeout -k 10 240 python -u tools/ab_flash.py 2>/dev/null \
    | sed "s/^{/{\"case\": \"$label\", /" >> "$OUT" || exit $?
done

#!/usr/bin/env bash
# Recreate the importable reference used ONLY to generate golden fixtures
# (tests/golden/make_golden.py).  Runs in the build container, never on the
# GPU box.  The reference is Python 2; this converts a scratch copy in /tmp to
# Python 3 mechanically.  Nothing is copied into the repo.
set -euo pipefail
DST=${1:-/tmp/oracle}
SRC=/root/reference/hyperopt
[ -d "$SRC" ] || { echo "reference not present at $SRC" >&2; exit 1; }
rm -rf "$DST" && mkdir -p "$DST"
cp -r "$SRC" "$DST/"
cd "$DST"
python3 -m lib2to3 -w -n hyperopt > "$DST/2to3.log" 2>&1
sed -i -E 's/\basync\b/async_/g' hyperopt/base.py hyperopt/fmin.py hyperopt/mongoexp.py hyperopt/ipy.py
sed -i 's/    order = nx.topological_sort(G)/    order = list(nx.topological_sort(G))/' hyperopt/pyll/base.py
PYTHONPATH="$DST" python3 -c "import hyperopt, hyperopt.tpe" && echo "reference importable at $DST"

#!/bin/bash
# Reproduces the round-5 engine-actor hang (gpurun_out/r05u_test.log: pytest
# timeout inside fnnue_backend_go) on the CPU: the host pool of workers.h with
# one notify_one per ticket (the uncommitted pool of that run) against the
# committed notify_all, both driving tests/sanitize/workers_stress.cpp.
# Prints one line per run: the variant, its exit code (124 = hung, killed by
# the 60 s limit).
set -u
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/fishnet_amd/csrc" "$T/tests/sanitize"
python3 - "$ROOT/fishnet_amd/csrc/workers.h" "$T/fishnet_amd/csrc/workers.h" <<'PY'
import sys
s = open(sys.argv[1]).read()
a = "    cv_.notify_all();\n    work();"
assert a in s
open(sys.argv[2], "w").write(s.replace(a, "    for (size_t i = 0; i < want; ++i) cv_.notify_one();\n    work();"))
PY
cp "$ROOT/tests/sanitize/workers_stress.cpp" "$T/tests/sanitize/"
g++ -std=c++17 -O2 -pthread "$T/tests/sanitize/workers_stress.cpp" -o "$T/notify_one"
g++ -std=c++17 -O2 -pthread "$ROOT/tests/sanitize/workers_stress.cpp" -o "$T/notify_all"
for v in notify_one notify_all; do
  for i in 1 2 3; do
    timeout 60 "$T/$v" > /dev/null
    echo "$v run $i rc=$?"
  done
done
rm -rf "$T"

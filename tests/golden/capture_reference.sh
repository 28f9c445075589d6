#!/usr/bin/env bash
# Golden-fixture generator: runs the reference's own policy/demand scripts
# (read-only, from /root/reference) UNMODIFIED under bash, with the stub
# kubectl/aws/pkill/lsof of tests/golden/stubs on PATH, and records every
# payload they hand to kubectl into tests/golden/reference_capture/<variant>/.
#
# The scripts are copied to a scratch dir under /tmp to run (they source
# ./demo_00_env.sh relative to the cwd); nothing from the reference is copied
# into the repository -- only the payloads the scripts emit (data).
#
# Scripts exercised:
#   demo_19_reset_policies.sh   (RESET_KILL_PF=false: no process is signalled)
#   demo_10_setup_configure.sh  (PDB + pool labels)
#   demo_20_offpeak_configure.sh, demo_21_peak_configure.sh (NodePool patches)
#   demo_30_burst_configure.sh  (burst Deployments)
set -euo pipefail
REF="${REF:-/root/reference}"
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/reference_capture"
STUBS="$HERE/stubs"
[ -d "$REF" ] || { echo "reference not present at $REF" >&2; exit 2; }
chmod +x "$STUBS"/*
rm -rf "$OUT"; mkdir -p "$OUT"

run_variant() {   # run_variant <name> <script> [VAR=value ...]
  local name="$1" script="$2"; shift 2
  local cap="$OUT/$name"; mkdir -p "$cap"
  local work; work="$(mktemp -d /tmp/ccka_refcap.XXXXXX)"
  cp "$REF"/demo_00_env.sh "$REF/$script" "$work/"
  rm -f /tmp/np_req_*.json
  # the script's status is recorded, not trapped by set -e
  local rc=0
  ( cd "$work" && env -i HOME="$HOME" PATH="$STUBS:/usr/bin:/bin" CAPTURE_DIR="$cap" \
      RESET_KILL_PF=false "$@" bash "./$script" > "$cap/stdout.txt" 2> "$cap/stderr.txt" ) || rc=$?
  echo "$rc" > "$cap/exit_code"
  rm -f "$cap/.seq" /tmp/np_req_*.json
  rm -rf "$work"
}

run_variant reset_default      demo_19_reset_policies.sh
run_variant setup_default      demo_10_setup_configure.sh
run_variant offpeak_default    demo_20_offpeak_configure.sh
run_variant peak_default       demo_21_peak_configure.sh
run_variant burst_default      demo_30_burst_configure.sh
run_variant offpeak_two_zones  demo_20_offpeak_configure.sh OFFPEAK_ZONES=us-east-2a,us-east-2b
run_variant offpeak_empty_env  demo_20_offpeak_configure.sh OFFPEAK_ZONES=
run_variant peak_space_zones   demo_21_peak_configure.sh "PEAK_ZONES=us-east-2b us-east-2c"
run_variant offpeak_custom_np  demo_20_offpeak_configure.sh NP_SPOT=cheap-pool NP_OD=slo-pool
run_variant burst_small        demo_30_burst_configure.sh COUNT=3 REPLICAS=2 NAMESPACE=ns-small
# keep stdout banners out of the fixtures except the exit codes (they print env values)
# mktemp names are random: normalise them so the fixtures are reproducible
find "$OUT" -name kubectl_argv.log -exec sed -i -E 's#/tmp/(burst-web\.yaml|np_req)[^ ]*#/tmp/<tmpfile>#g' {} +
find "$OUT" -name stdout.txt -delete
find "$OUT" -name stderr.txt -delete
( cd "$OUT" && find . -type f | sort | xargs sha256sum ) > "$HERE/reference_capture.sha256"
echo "captured into $OUT"

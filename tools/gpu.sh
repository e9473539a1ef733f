#!/bin/bash
# Parameterised GPU session (one gpurun call; replaces the round-3 one-off scripts).
# Each argument is one step, run in order:
#   tests:<pytest args>                  pytest -m gpu on the given files / -k filters
#   bench:<tag>[:<ENV=V,...>][:<bench.py args>]
#                                        bench.py -> gpurun_out/<tag>.json (+ .err)
#   prof:<tag>[:<ENV=V,...>][:<bench.py args>]
#                                        rocprofv3 --kernel-trace --stats (csv) of bench.py
#   pmc:<tag>:<COUNTER+COUNTER...>[:<bench.py args>]
#                                        one rocprofv3 --pmc pass (counters of one pass only)
#   pmce:<tag>:<ENV=V,...>:<COUNTER+...>[:<bench.py args>]   the same with environment settings
#   py:<tag>:<script and args>           python -u <script args> -> gpurun_out/<tag>.txt
#   smoke                                __graft_entry__.smoke()
# Every step runs under its own time limit; a step that crashes, times out or fails stops
# the session (pytest exit 1 = test failures: the session goes on).
#   gpurun --timeout 900 -- 'bash tools/gpu.sh "tests:tests/test_gpu_tb.py" "bench:b1::--no-extra"'
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ROOT=$(pwd)
envset() {  # ENV=V,ENV2=V2 -> exported
  local IFS=,
  for kv in $1; do [ -n "$kv" ] && export "$kv"; done
}
run_step() {
  local spec=$1 kind rest tag envs args rc
  kind=${spec%%:*}
  rest=${spec#*:}
  [ "$rest" = "$spec" ] && rest=""
  case $kind in
    tests)
      echo "=== tests $rest"
      timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread \
        $rest > gpurun_out/tests_$(date +%H%M%S).log 2>&1
      rc=$?
      echo "=== tests rc=$rc"
      tail -n 25 "$(ls -t gpurun_out/tests_*.log | head -n 1)" | cut -c1-300
      [ $rc -le 1 ] && return 0 || return $rc ;;
    bench|prof)
      tag=${rest%%:*}; rest=${rest#"$tag"}; rest=${rest#:}
      envs=${rest%%:*}; args=${rest#"$envs"}; args=${args#:}
      ( envset "$envs"
        if [ "$kind" = bench ]; then
          timeout -k 10 600 python bench.py $args > gpurun_out/$tag.json 2> gpurun_out/$tag.err
        else
          cd /tmp && export TMPDIR=/tmp
          timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$ROOT/gpurun_out/$tag" -o run -- python3 "$ROOT/bench.py" $args \
            > "$ROOT/gpurun_out/$tag.log" 2>&1
        fi )
      rc=$?
      echo "=== $kind $tag ($envs) rc=$rc"
      [ "$kind" = bench ] && head -c 600 gpurun_out/$tag.json && echo && tail -n 3 gpurun_out/$tag.err
      return $rc ;;
    pmc|pmce)
      tag=${rest%%:*}; rest=${rest#"$tag"}; rest=${rest#:}
      envs=""
      if [ "$kind" = pmce ]; then envs=${rest%%:*}; rest=${rest#"$envs"}; rest=${rest#:}; fi
      local ctr=${rest%%:*}; args=${rest#"$ctr"}; args=${args#:}
      ( envset "$envs"
        cd /tmp && export TMPDIR=/tmp
        timeout -s KILL 300 rocprofv3 --pmc ${ctr//+/ } --output-format csv \
          -d "$ROOT/gpurun_out/$tag" -o run -- python3 "$ROOT/bench.py" $args \
          > "$ROOT/gpurun_out/$tag.log" 2>&1 )
      rc=$?
      echo "=== pmc $tag ($ctr) rc=$rc"
      return $rc ;;
    py)
      tag=${rest%%:*}; args=${rest#"$tag"}; args=${args#:}
      timeout -k 10 600 python -u $args > gpurun_out/$tag.txt 2>&1
      rc=$?; echo "=== py $tag rc=$rc"; tail -n 12 gpurun_out/$tag.txt | cut -c1-300
      return $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
      rc=$?; echo "=== smoke rc=$rc"; return $rc ;;
    *)
      echo "unknown step $spec"; return 2 ;;
  esac
}
for spec in "$@"; do
  run_step "$spec" || exit $?
done
exit 0

# Per-(config, op) evidence pass: one cold bench line, a rocprofv3 kernel
# trace (--stats), FETCH_SIZE and WRITE_SIZE in separate --pmc passes, and
# one SQ pass (8 counters), all of the same `bench.py --op` command.
#   SPECS="C3:decode C5:decode M:get" bash tools/prof_ops.sh
# Output under gpurun_out/p3/<cfg>_<op>*; tools/prof_collect.py summarises.
set -u
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/p3"
# the product-tree hash these counters describe (bench.py compares it with its own)
(cd "$R" && python3 -c "import bench; print(bench.product_tree_hash())") > "$R/gpurun_out/p3/product_tree.txt"
STEPS=${STEPS:-20}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM"
for spec in ${SPECS}; do
  c=${spec%%:*}; op=${spec##*:}; o="$R/gpurun_out/p3/${c}_${op}"
  B="$R/bench.py --config $c --op $op --no-cpu --no-host --passes 1 ${BARGS:-}"
  cd "$R"
  echo "$(date +%T) $c $op line"
  timeout -k 10 300 python3 $B --steps $STEPS > "$o.line.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "line $c $op rc=$rc"; tail -5 "$o.line.log"; exit $rc; }
  grep '^{' "$o.line.log" | tail -1
  [ "${PROF:-1}" = 1 ] || continue
  cd /tmp && export TMPDIR=/tmp
  echo "$(date +%T) $c $op trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${o}_trace" -o run --output-format csv -- python3 $B --steps $STEPS --warmup 3 --no-warm > "$o.trace.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "trace $c $op rc=$rc"; exit $rc; }
  for pass in FETCH_SIZE WRITE_SIZE SQ; do
    cnt=$pass; [ $pass = SQ ] && cnt=$SQ
    echo "$(date +%T) $c $op $pass"
    timeout -s KILL 240 rocprofv3 --pmc $cnt -d "${o}_$pass" -o run --output-format csv -- python3 $B --steps 8 --warmup 2 --no-warm > "$o.$pass.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $pass $c $op rc=$rc"; exit $rc; }
  done
done
exit 0

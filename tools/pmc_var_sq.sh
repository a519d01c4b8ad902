# One SQ counter pass (CNT, <= 8 SQ counters) of `bench.py --config $CFG --op $OP`
# per library variant in VARS (head = in-tree; else abl/libpackos_<v>.so).
set -u
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmcv"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/pmcv/avail.txt" 2>&1; echo "list rc=$?"
for v in ${VARS:-head}; do
  L=""; [ "$v" = head ] || L="$R/abl/libpackos_$v.so"
  PACKOS_LIB=$L timeout -s KILL 120 rocprofv3 --pmc ${CNT} -d "$R/gpurun_out/pmcv/${CFG}_${OP}_$v" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --op $OP --steps 6 --warmup 2 --no-warm --no-cpu --no-host > "$R/gpurun_out/pmcv/${CFG}_${OP}_$v.log" 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/pmcv/${CFG}_${OP}_$v.log"; exit $rc; }
done

# Kernel-trace stats of one weight-gradient op (OP args) at several persistent grid sizes, plus one PMC pass.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OPARGS=${OPARGS:-"wgrad 256 32 32 64 32 30"}
cd /tmp
for nb in ${GRIDS:-256 128 512}; do
  rm -rf $R/gpurun_out/wg_$nb
  HLMC_WGRAD_HALO_BLOCKS=$nb timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wg_$nb -o run --output-format csv -- python3 $R/scripts/op_probe.py $OPARGS > $R/gpurun_out/wg_$nb.log 2>&1 || { echo "trace $nb failed"; exit 1; }
  f=$(find $R/gpurun_out/wg_$nb -name "*kernel_stats.csv" | head -1)
  echo "== blocks $nb"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(f\"{float(r['AverageNs'])/1e3:8.2f} us x{r['Calls']:>4}  {r['Name'][:110]}\")
"
done
rm -rf $R/gpurun_out/wg_pmc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/wg_pmc -o run --output-format csv -- python3 $R/scripts/op_probe.py $OPARGS > $R/gpurun_out/wg_pmc.log 2>&1; echo "pmc rc=$?"
f=$(find $R/gpurun_out/wg_pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'][:60]; acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    print(k); print('   ', {c: round(v) for c, v in d.items()})
PY

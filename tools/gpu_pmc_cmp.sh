set -o pipefail
cd "$GRAFT_REPO_ROOT"
PMC_ROLL=1 timeout -k 10 500 bash tools/pmc.sh r3_pmc_lag2 > /dev/null || exit 1
GSM_LIB_PATH=$GRAFT_REPO_ROOT/gs-marl_amd/gsmarl_amd/lib/ablate/graph.so PMC_ROLL=1 timeout -k 10 500 bash tools/pmc.sh r3_pmc_lb > /dev/null || exit 1
for t in lag2 lb; do python - <<PY
import json
t=open('gpurun_out/r3_pmc_$t/summary.txt').read(); d=json.loads(t[t.index('{'):])
c=d['roll']['counters']; w=c['SQ_WAVES']
print('$t', 'valu/w', round(c['SQ_INSTS_VALU']/w/100,1), 'salu/w', round(c['SQ_INSTS_SALU']/w/100,1), 'lds/w', round(c['SQ_INSTS_LDS']/w/100,1),
 'wave_cyc', c['SQ_WAVE_CYCLES'], 'wait_any', round(c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES'],3), 'wait_inst', round(c['SQ_WAIT_INST_ANY']/c['SQ_WAVE_CYCLES'],3), 'active', round(c['SQ_ACTIVE_INST_ANY']/c['SQ_WAVE_CYCLES'],3), 'gui', c['GRBM_GUI_ACTIVE'])
PY
done

#!/bin/bash
# FETCH_SIZE calibration for 4 / 8 / 16 B-per-lane coalesced reads (tools/fetch_calib.hip), one --pmc pass.
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r06_fetch_calib -o run --output-format csv \
  -- $R/tools/_bin/fetch_calib > $R/gpurun_out/r06_fetch_calib.log 2>&1
rc=$?; echo "calib rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/r06_fetch_calib/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Kernel_Name'][:70], r['Counter_Name'], round(float(r['Counter_Value']) * 1024 / 2**30, 4), 'GiB of 1 GiB read')
PY

#!/bin/bash
# FETCH_SIZE calibration by access width (tools/pmc_calib.hip): one rocprofv3 --pmc pass, then per kernel
# FETCH_SIZE x 1024 / bytes read.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_calib -o calib --output-format csv -- $R/tools/_build/pmc_calib || exit $?
python3 - "$R/gpurun_out/pmc_calib" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
name = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        d = int(row["Dispatch_Id"])
        per[d] += float(row["Counter_Value"])
        name[d] = row["Kernel_Name"].split("(")[0]
by = collections.defaultdict(list)
for d in sorted(per):
    by[name[d]].append(per[d])
for k, v in by.items():
    print(k, "FETCH_SIZE KiB per dispatch", v, "ratio FETCH_SIZE bytes / bytes read", [round(x * 1024 / 2**30, 4) for x in v])
PY

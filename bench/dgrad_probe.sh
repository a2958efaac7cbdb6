#!/bin/bash
# Run bench/dgrad_probe.py on the probe variant library (abso/so_probe.so, built with
# PMD_EXTRA_CFLAGS=-DPMD_DGRAD_PROBE=1 python csrc/build.py --variant probe); the production
# library is restored afterwards.  Arguments go to dgrad_probe.py.
set -u
export PMD_NO_AUTOBUILD=1
export PMD_ALLOW_VARIANT=1
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abso/so_prod_backup.so
cp abso/so_probe.so $SO
python bench/dgrad_probe.py "$@"
rc=$?
cp abso/so_prod_backup.so $SO
exit $rc

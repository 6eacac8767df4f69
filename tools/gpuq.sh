#!/bin/bash
# retry a gpurun call only while the pool has no free slot/box (exit code 3); any other outcome ends it
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 60
done
exit 3

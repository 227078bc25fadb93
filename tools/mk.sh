#!/bin/bash
# build everything in-tree; print errors / warnings and fail on any error (dev helper)
cd "$(dirname "$0")/.." || exit 1
make -j8 -C semi-direct-visual-odometry_amd > /tmp/mk.log 2>&1
rc=$?
grep -E "error|warning" /tmp/mk.log | head -30
exit $rc

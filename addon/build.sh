#!/bin/sh
# Build the Node-API addon (C) against the system Node headers, linked to the in-tree libgbv.so.
set -e
cd "$(dirname "$0")"
NODE_INC=${NODE_INC:-/usr/include/node}
gcc -O2 -fPIC -shared -pthread -Wall -Wextra -Wno-unused-parameter -I"$NODE_INC" -o gbv_addon.node.tmp gbv_addon.c \
    -L../lodestar_amd -lgbv -Wl,-rpath,'$ORIGIN/../lodestar_amd'
mv gbv_addon.node.tmp gbv_addon.node

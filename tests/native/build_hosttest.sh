#!/bin/sh
# Host-only build of the device arithmetic headers for CPU unit tests (not a product path).
set -e
cd "$(dirname "$0")"
hipcc -O2 -fPIC -shared --offload-host-only -o libhosttest.so hosttest.cpp

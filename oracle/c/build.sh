#!/bin/sh
# Build the CPU port (test/bench infrastructure; see blsport.c header).
set -e
cd "$(dirname "$0")"
gcc -O3 -march=x86-64-v3 -fPIC -shared -pthread -Wall -Wno-unused-function -o libblsport.so blsport.c

#!/bin/bash
# builds scripts/lr_phases.cpp against the in-tree libraries (run `make` first)
R=$(cd $(dirname $0)/.. && pwd)
g++ -std=c++17 -O2 -I$R/include -I$R/aby3_amd/host $R/scripts/lr_phases.cpp -o $R/scripts/lr_phases \
    -L$R/aby3_amd/lib -laby3 -laby3gpu -Wl,-rpath,$R/aby3_amd/lib -pthread

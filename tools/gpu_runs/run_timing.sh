#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/phase_timing.py > gpurun_out/timing.log 2>&1; rc=$?; cat gpurun_out/timing.log | tail -40; exit $rc

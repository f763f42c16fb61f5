#!/bin/bash
# the cadence sweep of DESIGN.md §3d on the CPU oracle (64 and 8 hosts x 8 services, 3000 rounds)
cd "$(dirname "$0")/../.."
for a in '8 8 3000 1 15 100 {}' '8 8 3000 1 15 100 {"push_pull_stagger":1}' \
         '64 8 3000 1 15 100 {}' '64 8 3000 0 15 100 {}' '64 8 3000 1 15 100 {"push_pull_stagger":1}' \
         '64 8 3000 1 15 100 {"push_pull_stagger":1,"probe_piggyback":1}' '64 8 3000 1 15 200 {"push_pull_stagger":1}' \
         '64 8 3000 1 15 20 {}' '64 8 3000 1 15 10 {}' '64 8 3000 1 1 100 {}' '64 8 3000 1 1 100 {"push_pull_stagger":1,"probe_piggyback":1}'; do
  python profiles/r06/trace_small.py $a
done

#!/bin/bash
# Round 5: the union's row lookup through a 64-entry slot table (tree) against the cached-rows
# build (build_ab/cache).
AB=cache bash profiles/r05/call_ae.sh ${1:-r05ap}

#!/bin/bash
# Round-4 last tree: every GPU test and smoke (r04_final_tests.sh), then the bench line and the
# rocprofv3 kernel stats of a short bench run (r04_meas2.sh), on one box.
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/r04_final_tests.sh r04_last && bash tools/gpu/r04_meas2.sh r04_last

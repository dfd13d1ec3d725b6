# rocprof kernel traces: config-4 bench and the rank-0-of-8 proxy
set -e
bash tools/prof_full.sh r6a
bash tools/prof_emul.sh r6a

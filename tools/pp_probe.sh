set -e
for f in --no-defer --native-sum; do echo "== $f"; PYTHONPATH=. timeout -k 10 200 python tools/side_probe.py --capture-first $f 2>&1 | grep -v Warn | tail -4; done

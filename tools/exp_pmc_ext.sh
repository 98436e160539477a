export TMPDIR=/tmp
mkdir -p gpurun_out/pe
for m in 1 2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    BSQ_TEST_EXT_NEST=$m timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pe/m${m}_$c -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > gpurun_out/pe/m${m}_$c.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob
for m in (1, 2):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        tot = 0.0
        for f in glob.glob(f"gpurun_out/pe/m{m}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_extend" in r["Kernel_Name"]:
                    tot += float(r["Counter_Value"]) * 1024
        print(m, c, round(tot / 1e9, 4), "GB per 1M-read lone launch", flush=True)
PY

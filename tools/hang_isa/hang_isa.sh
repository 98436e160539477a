#!/bin/bash
# CPU only: gfx950 ISA of klib's partition scan `do ++i; while (lt(a[i], rp))` over lane-interleaved scratch,
# unbounded (klib as written, -DBSQ_INTROSORT_UNBOUNDED) and bounded (`i < t &&`, the shipping form), in
#   * the probe kernel (introsort_probe.hip: sort_dedup_patch's sort by `re` over SP<int, 64> / S = 1 scratch) and
#   * k_extend<true, 64> itself (instantiated only under BSQ_ISA_PROBE).
# Prints each build's scan loop: the load of a[i + 1] (offset:256 = one element of a 64-lane-interleaved int array),
# the load of that element's `re` and the exit compare.  Output files under /tmp/hang_isa.
set -e
here=$(cd "$(dirname "$0")" && pwd)
out=/tmp/hang_isa; mkdir -p $out
for v in bounded unbounded; do
  extra=""; [ $v = unbounded ] && extra="-DBSQ_INTROSORT_UNBOUNDED"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBSQ_ISA_PROBE $extra --cuda-device-only -S \
      -o $out/all_$v.s "$here/introsort_probe.hip"
  for k in k_introsort_probeILi64EE k_extendILb1ELi64EE; do
    s=$(grep -n "^_ZN3bsq[0-9]*${k}.*:" $out/all_$v.s | head -1 | cut -d: -f1)
    e=$(awk -v s=$s 'NR > s && /^\.Lfunc_end/ {print NR; exit}' $out/all_$v.s)
    sed -n "${s},${e}p" $out/all_$v.s > $out/${k}_$v.s
    echo "== $v $k: first scan loop (of $(grep -c 'off offset:256$' $out/${k}_$v.s) a[i+1] loads)"
    grep -n -B1 -A11 'global_load_dword v[0-9]*, v\[[0-9:]*\], off offset:256$' $out/${k}_$v.s | head -14
  done
done

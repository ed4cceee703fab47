set -o pipefail
for shp in "4 48 64" "64 256 256" "4 481 321" "2 37 29"; do
  PSGLA_LIB=exp_libs/lib_barc.so timeout -k 10 60 python3 tools/bar_probe.py $shp > gpurun_out/bar_$$.txt 2>&1 || { cat gpurun_out/bar_$$.txt; exit 1; }
  tail -1 gpurun_out/bar_$$.txt
  grep -q " 0 with unequal" gpurun_out/bar_$$.txt || { cat gpurun_out/bar_$$.txt; exit 1; }
done

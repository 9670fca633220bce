set -eo pipefail
OUT=gpurun_out/r03s; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "demand or two_levels or default_on" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
FAC_LIB=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_prof.so FAC_DIAGNOSTICS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.err
grep FAC_PROF $OUT/prof.err | tail -4
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err; cut -c1-400 $OUT/c3.json
timeout -k 10 400 python bench.py --vocab 0 --no-cpu-baseline > $OUT/c3_vocab0.json 2> $OUT/c3_vocab0.err; cut -c1-400 $OUT/c3_vocab0.json
timeout -k 10 400 python bench.py --config c2 --vocab 0 --no-cpu-baseline > $OUT/c2_vocab0.json 2> $OUT/c2_vocab0.err; cut -c1-400 $OUT/c2_vocab0.json

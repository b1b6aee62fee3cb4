bash tools/gpu.sh r05zc \
 'tA|500|python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_source_net.py -q -rx --timeout 300 --timeout-method thread -p no:cacheprovider' \
 'tB|500|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --ignore=tests/test_gpu_configs.py --ignore=tests/test_gpu_net.py --ignore=tests/test_gpu_source_net.py' \
 'smoke|200|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")"'

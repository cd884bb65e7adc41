# knob-path parity tests (association, step 12b)
export O=gpurun_out/r07z
PYTEST_K="knob_paths" bash tools/gpu.sh tests

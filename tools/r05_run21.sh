# closing-HEAD checks: full GPU suite, smoke, default bench line (C2 + C3 roofline + live path + CPU baseline)
export O=gpurun_out/r07x
bash tools/gpu.sh tests smoke bench

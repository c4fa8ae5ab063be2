# chunks of 4 on the whole 1080p C4 frame by default: the ReSTIR / C4 parity tests, the GPU suite
# rest (-x over everything), smoke and the default bench line
bash tools/gpu_suite.sh r05q

for d in 0 1 2 3; do echo "--- diag=$d"; GGML_MI355X_DIAG=$d timeout -k 10 120 python scripts/stamps_probe.py q4_0 4096 4096 1 2>&1 | grep -v amdgpu; done
for d in 0 1; do echo "--- diag=$d"; GGML_MI355X_DIAG=$d timeout -k 10 120 python scripts/stamps_probe.py q4_K 4096 11008 1 2>&1 | grep -v amdgpu; done

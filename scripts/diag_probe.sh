for t in q4_0 q4_K q5_K q6_K; do
  for d in 0 2; do echo "--- diag=$d"; GGML_MI355X_DIAG=$d timeout -k 10 120 python scripts/stamps_probe.py $t 4096 4096 1 16 2>&1 | grep -v amdgpu; done
done

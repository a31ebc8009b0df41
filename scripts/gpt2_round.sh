set -u
scripts/gpt2_iter.sh || exit 1
scripts/gpt2_ab.sh head nopf || exit 1
CFGS="GGML_MI355X_LAYER_FUSION=1 GGML_MI355X_LAYER_FUSION=0" scripts/plugin_gpt2_ab.sh

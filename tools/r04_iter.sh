# (transitional alias while an in-flight run uses the old name)
ROUND=r04 bash tools/gpu_iter.sh

# Round-5 call: pace thresholds (gsm_device.h pace_level variants: t2 / t6 =
# a quarter / three quarters of a step instead of a half, l4 = a fourth
# level) against the library, same box, driver and h lines.
cd $GRAFT_REPO_ROOT
AB_LINES="driver h" bash tools/gpu.sh ab cq t2 t6 l4 || exit 5

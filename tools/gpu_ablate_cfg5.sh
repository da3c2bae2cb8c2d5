# cfg5 ATE ablations: the TrackSIM cfg5 stream for 300 frames with one factor changed at a
# time; one bench line each (ate_rmse_m).   usage: bash tools/gpu_ablate_cfg5.sh TAG [workload]
set -e
TAG=${1:-abl}
WL=${2:-cfg5}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
B="python -u bench.py --workload $WL --steps 300 --cpu-frames 0 --no-host-feed"
run() { name=$1; shift; timeout -k 10 240 $B "$@" > $O/$name.json 2> $O/$name.err; }
run base
run no_uwb --set use_uwb=0 --sim uwb=false
run anchors_fixed --set anchors_fix=1
run no_imu_intr --set do_calib_imu_intrinsics=0 --set do_calib_imu_g_sensitivity=0
run no_imu_intr_no_uwb --set do_calib_imu_intrinsics=0 --set do_calib_imu_g_sensitivity=0 --set use_uwb=0 --sim uwb=false
run two_cams --set num_cameras=2
run no_cam_calib --set do_calib_camera_pose=0 --set do_calib_camera_intrinsics=0 --set do_calib_camera_timeoffset=0
run ideal_imu --sim noisy_imu=false
run ideal_imu_no_uwb --sim noisy_imu=false --set use_uwb=0 --sim uwb=false
python - $O <<'PY'
import json, os, sys
o = sys.argv[1]
for f in sorted(os.listdir(o)):
    if f.endswith(".json"):
        try:
            d = json.loads(open(os.path.join(o, f)).read().strip().splitlines()[-1])
            print("%-22s ate %.4f m  ori %.3f deg  frames/s %.1f  msckf %.0f" % (f[:-5], d["ate_rmse_m"], d["ate"]["ori_rmse_deg"], d["value"], d["config"]["mean_msckf_feats"]))
        except Exception as e:
            print(f, "failed", e)
PY

# round-4 session R: walk length per wave-chunk (m = 13 planner / 14 / 15) on the bench and near-dense matrices
bash tools/gpu_session.sh r4r "walklen=python3 tools/probe_walklen2.py 0 14 15 0 14 15"

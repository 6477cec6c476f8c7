# second-stream priority A/B (EngineOptions.side_priority), with the device's range printed first
cd "$(dirname "$0")/../.."
python3 -c "import torch; print('priority range (low, high):', torch.cuda.Stream.priority_range())" || exit 1
lo=$(python3 -c "import torch; print(torch.cuda.Stream.priority_range()[0])")
hi=$(python3 -c "import torch; print(torch.cuda.Stream.priority_range()[1])")
bash tools/gpu_ab_engine.sh prio "{\"side_priority\":$lo}" "{\"side_priority\":$hi}" "{\"wn_bwd_split\":true}"

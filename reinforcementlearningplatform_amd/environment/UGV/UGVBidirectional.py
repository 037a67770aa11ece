"""UGVBidirectional — environment/UGV/UGVBidirectional.py on MI355X (variant 'ppo2': the PPO2
demo copy's |e| gate on the heading term)."""
from ... import _abi
from .UGVForward import UGVForward


class UGVBidirectional(UGVForward):
    KIND = _abi.RLP_ENV_UGV_BIDIRECTIONAL

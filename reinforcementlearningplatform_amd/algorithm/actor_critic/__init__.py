"""Off-policy actor-critic algorithms (algorithm/actor_critic/ of the reference)."""

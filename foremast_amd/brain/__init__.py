"""The brain: GPU streaming engine and the job loop."""

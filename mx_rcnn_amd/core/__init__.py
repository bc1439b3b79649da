"""Training / evaluation runtime: flat params, trainer (MutableModule-style API), metrics,
callbacks, LR schedules, hipGraph step capture, detector / tester."""

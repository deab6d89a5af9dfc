"""Minimal goal-pose container with the attribute surface of the reference's
``utils/pose.py:4-112`` that the solver API exposes (``target_pose.pose`` xyz,
``target_pose.orientation`` quaternion **xyzw**, ``clone``)."""
import torch


class Pose:
    def __init__(self):
        self.pose = torch.zeros(3)
        self.orientation = torch.tensor([0.0, 0.0, 0.0, 1.0])

    @property
    def np_pose(self):
        return self.pose.numpy()

    @property
    def np_orientation(self):
        return self.orientation.numpy()

    def clone(self):
        p = Pose()
        p.pose = self.pose.clone()
        p.orientation = self.orientation.clone()
        return p

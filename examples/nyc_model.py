"""The NYC taxi fare MLP shared by the examples (reference: NYC_Model in
examples/pytorch_nyctaxi.py, raytrain_nyctaxi.py, horovod_nyctaxi.py)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class NYC_Model(nn.Module):
    def __init__(self, cols):
        super().__init__()
        self.fc1, self.fc2, self.fc3 = nn.Linear(cols, 256), nn.Linear(256, 128), nn.Linear(128, 64)
        self.fc4, self.fc5 = nn.Linear(64, 16), nn.Linear(16, 1)
        self.bn1, self.bn2, self.bn3, self.bn4 = (nn.BatchNorm1d(256), nn.BatchNorm1d(128),
                                                  nn.BatchNorm1d(64), nn.BatchNorm1d(16))

    def forward(self, *x):
        x = torch.cat(x, dim=1) if len(x) > 1 else x[0]
        x = self.bn1(F.relu(self.fc1(x)))
        x = self.bn2(F.relu(self.fc2(x)))
        x = self.bn3(F.relu(self.fc3(x)))
        x = self.bn4(F.relu(self.fc4(x)))
        return self.fc5(x)

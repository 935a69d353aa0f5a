"""Drop-in for the reference's ``epoch_dataloader.py`` (VideoDataset, lines 7-33).

``__getitem__`` returns ``{'video': [T,3,224,224] f32, 'label': [1] f32}`` like the reference,
built by this package's ``utils.get_video_from_video_info`` (JPEG decode on the host, crop /
flip / normalise by ``eosv_crop_normalize_frames``; offline, the synthetic frame generator), so
the video is already a DEVICE tensor.  A ``DataLoader`` over it must therefore run in the main
process (``num_workers=0``): CUDA cannot be initialised in forked workers.
"""
import torch
from torch.utils.data import Dataset

from utils import get_label_from_video_info, get_video_from_video_info


class VideoDataset(Dataset):
    def __init__(self, info_txt, root_dir, mode='train', data_aug=None, transform=None):
        self.info_txt = info_txt
        self.root_dir = root_dir
        self.mode = mode
        self.data_aug = data_aug
        self.transform = transform
        self.info_list = open(self.info_txt).readlines()

    def __len__(self):
        return len(self.info_list)

    def __getitem__(self, idx):
        video_info = self.info_list[idx].strip('\n')
        video = get_video_from_video_info(video_info, mode=self.mode, frame_dir=self.root_dir, data_aug=self.data_aug)
        video_label = get_label_from_video_info(video_info, self.info_txt)
        return {'video': video.float(), 'label': torch.FloatTensor([int(video_label)])}

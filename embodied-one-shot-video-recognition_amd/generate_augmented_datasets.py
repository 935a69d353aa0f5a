"""Drop-in for the gallery helpers of the reference's ``generate_augmented_datasets.py``
(lines 4-36), which ``network_test.py`` imports under its old name
``generate_gallery_videos`` (network_test.py:21).

The offline "trainAug 2.3" dataset writer (generate_augmented_datasets.py:38-186:
shell ``cp`` of frame directories, broken as shipped) is training-data generation,
outside the test-time path, and is not provided.
"""
import random

import torch

import utils


def generate_gallery_list(num=10):
    """generate_augmented_datasets.py:4-23 -- ``num`` random train videos per class
    (global RNG, class order of first appearance) written to utils.GALLERY_LIST."""
    data = open(utils.TRAIN_LIST).readlines()
    groups = {}
    for line in data:
        line = line.strip('\n')
        groups.setdefault(line.split('/')[0], []).append(line)
    with open(utils.GALLERY_LIST, 'w') as f:
        for cname in groups.keys():
            for info in random.sample(groups[cname], num):
                print(info, file=f)


def gallery_video_infos():
    return [line.strip('\n') for line in open(utils.GALLERY_LIST).readlines()]


def generate_gallery_videos():
    """generate_augmented_datasets.py:25-36 -> [G,16,3,224,224] f32 (host)."""
    videos = [utils.get_video_from_video_info(vi, mode='test') for vi in gallery_video_infos()]
    return torch.stack(videos)

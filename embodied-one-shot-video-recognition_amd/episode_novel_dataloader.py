"""Drop-in for the reference's ``episode_novel_dataloader.py`` (lines 4-80).

``EpisodeDataloader(mode).get_episode()`` returns the same dict as the reference
(support_x [n*k,T,3,224,224] f32, support_y [n*k] f32, query_x [1,<=T,3,224,224] f32,
query_y [1] f32, support_x_frames list) and consumes the GLOBAL ``random`` module in
the reference's order, so ``random.seed(s)`` reproduces the reference's episodes.
``get_episode_plan()`` draws the same episode without loading frames; the batched
GPU path (network_test.py) uses it to keep frames on the device.
"""
import random

import torch

import utils
from eosv import episodes as _episodes


class EpisodeDataloader():
    '''
    get_episode: return episode
    shuffle label every episode
    '''

    def __init__(self, mode='test'):
        self.mode = mode
        if mode == 'train':
            self.dataset_list = utils.TRAIN_LIST
        elif mode == 'val':
            self.dataset_list = utils.VAL_LIST
        elif mode == 'test':
            self.dataset_list = utils.TEST_LIST
        self.data = open(self.dataset_list).readlines()
        self._index = _episodes.class_index(self.data)

    def get_episode_plan(self):
        """The RNG draws of get_episode (episode_novel_dataloader.py:34-70), no frames."""
        return _episodes.sample_episode(self._index, utils.n_way, utils.k_shot, random)

    def load_episode(self, plan):
        """Frames for a plan, exactly as the reference loads them (:45-80)."""
        T = utils.VIDEO_FRAMES
        support_x, support_x_frames = [], []
        for vi in plan['support']:
            v, n = utils.get_video_from_video_info_3(vi, mode=self.mode, video_frames=T)
            support_x.append(v)
            support_x_frames.append(n)
        query_x = [utils.get_video_from_video_info(plan['query'], mode='test', video_frames=T)]
        return {'support_x': torch.stack(support_x).float(),
                'support_y': torch.FloatTensor(plan['support_y']),
                'query_x': torch.stack(query_x).float(),
                'query_y': torch.FloatTensor([plan['query_y']]),
                'support_x_frames': support_x_frames}

    def get_episode(self):
        '''
        :return: support_x = n_way * k_shot * video, support_y = n_way * k_shot * y,;
        :return: query_x = 1* video , query_y = 1 * y
        '''
        if self.mode != 'train':  # loading draws nothing from the RNG outside train mode
            return self.load_episode(self.get_episode_plan())
        # train mode: frame loading draws from the RNG too, so interleave like :45-70
        T = utils.VIDEO_FRAMES
        d = self._index
        names = random.sample(tuple(d.keys()), utils.n_way)
        qname = random.sample(names, 1)[0]
        sx, sxf, sy, qx, qy = [], [], [], [], []
        for cname in names:
            if cname == qname:
                infos = random.sample(d[cname], utils.k_shot + 1)
                qx.append(utils.get_video_from_video_info(infos[0], mode='test', video_frames=T))
                qy.append(names.index(cname))
                infos = infos[1:]
            else:
                infos = random.sample(d[cname], utils.k_shot)
            for vi in infos:
                v, n = utils.get_video_from_video_info_3(vi, mode=self.mode, video_frames=T)
                sx.append(v)
                sxf.append(n)
                sy.append(names.index(cname))
        return {'support_x': torch.stack(sx).float(), 'support_y': torch.FloatTensor(sy),
                'query_x': torch.stack(qx).float(), 'query_y': torch.FloatTensor(qy),
                'support_x_frames': sxf}

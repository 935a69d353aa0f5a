"""Drop-in for the reference's ``network_train.py`` (TrainNetwork, lines 21-131).

Same constructor, ``finetune_model(data_aug, pre_model)`` semantics and loss-file format; the
step itself runs natively (eosv.train.NativeTrainer over csrc/train.hip and csrc/gemm_f32.hip): ResNet in
train mode with batch-statistics BN, the clip mean over T frames (:100, :110), fc,
CrossEntropyLoss, backward, SGD(momentum=0.9) with lr_1 on the convnet and lr_2 on the fc, and
StepLR(step_size, gamma=0.1) stepped at the start of every epoch as the reference does (:83-84:
epoch e trains at lr * 0.1 ** ((e + 1) // step_size)).  One checkpoint per epoch in the
reference's state_dict layout (:130-131).

Deviations a caller can see:
- the DataLoader runs in the main process (the dataset yields device tensors), so the random
  crops / flips are drawn from the main process's RNG instead of 8 workers' reseeded ones;
- the running loss is a Python float (the reference's ``loss.data[0]`` raises on PyTorch >= 0.5);
- the loss file is closed at the end.
"""
import os

import numpy as np
import torch
from torch.utils.data import DataLoader

from epoch_dataloader import VideoDataset
from eosv.train import NativeTrainer
from models import model_resnet18, model_resnet50
from utils import KINETICS_FRAME_DIR, TRAIN_LIST, TrainAugSegDatasets_DIR_2_3, num_classes_train


class TrainNetwork():
    def __init__(self, loss_path, ckp_path, epoch_nums, batch_size, lr_1, lr_2, lr_step_size=10,
                 resnet_model='resnet50', num_classes=num_classes_train):
        self.loss_path = loss_path
        self.ckp_path = ckp_path
        self.epoch_nums = epoch_nums
        self.batch_size = batch_size
        self.lr_1 = lr_1
        self.lr_2 = lr_2
        self.lr_step_size = lr_step_size
        self.resnet_model = resnet_model
        self.num_classes = num_classes
        if not os.path.exists(self.ckp_path):
            os.makedirs(self.ckp_path)
        if self.resnet_model == 'resnet18':
            self.mymodel = model_resnet18(num_classes=self.num_classes)
        elif self.resnet_model == 'resnet50':
            self.mymodel = model_resnet50(num_classes=self.num_classes)
        self.mymodel.train()
        self.mymodel.cuda()
        print('model loaded.')
        self.myDataset = VideoDataset(TRAIN_LIST, KINETICS_FRAME_DIR, mode='train')
        self.myDataloader = DataLoader(self.myDataset, batch_size=self.batch_size, shuffle=True, num_workers=0)

    def lr_at(self, epoch):
        """StepLR stepped before each epoch's batches (network_train.py:77-84)."""
        f = 0.1 ** ((epoch + 1) // self.lr_step_size)
        return self.lr_1 * f, self.lr_2 * f

    def finetune_model(self, data_aug='None', pre_model=None):
        file = open(self.loss_path, 'w')
        if pre_model:
            self.mymodel.load_state_dict(torch.load(pre_model, weights_only=True))
            print(pre_model, 'loaded.')
        if data_aug == 'None':
            dataset_train = VideoDataset(TRAIN_LIST, KINETICS_FRAME_DIR, mode='train')
        elif data_aug == 'aug_seg_T':
            dataset_train = VideoDataset(TRAIN_LIST, TrainAugSegDatasets_DIR_2_3, mode='train')
        else:
            print('data aug error.')
            file.close()
            return 0
        dataloader_train = DataLoader(dataset_train, batch_size=self.batch_size, shuffle=True, num_workers=0)
        trainer = NativeTrainer(self.resnet_model, self.num_classes, device=torch.cuda.current_device())
        trainer.load_state_dict(self.mymodel.state_dict())
        self.trainer = trainer
        for epoch in range(self.epoch_nums):
            lr_1, lr_2 = self.lr_at(epoch)
            running_loss = 0.0
            for i_batch, sample_batched in enumerate(dataloader_train):
                video, label = sample_batched['video'], sample_batched['label']
                video_shape = video.shape
                video = video.reshape(-1, video_shape[2], video_shape[3], video_shape[4])
                label = label.view((label.shape[0])).long()
                loss, output = trainer.step(video, label.cpu().numpy(), video_shape[1], lr_1, lr_2)
                predicted_y = np.argmax(output.cpu().numpy(), axis=1)
                accuracy = np.mean(label.cpu().numpy() == predicted_y)
                running_loss = running_loss + loss
                if i_batch % 50 == 49:
                    print('[%d, %5d] loss: %.3f accuracy: %.3f' % (epoch + 1, i_batch + 1, running_loss / 50, accuracy))
                    print('[%d, %5d] loss: %.3f accuracy: %.3f' % (epoch + 1, i_batch + 1, running_loss / 50, accuracy),
                          file=file)
                    running_loss = 0.0
            save_model_path = self.ckp_path + 'model' + str(epoch + 1) + '.pkl'
            torch.save(trainer.state_dict(), save_model_path)
        self.mymodel.load_state_dict(trainer.state_dict())
        file.close()

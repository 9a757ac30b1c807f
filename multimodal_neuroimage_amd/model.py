"""Hot-path subset of the reference's model.py — MI355X build.

Classes keep the reference names, `Class(**kwargs)` constructors (trainer.create_model,
trainer.py:176-266), forward signatures, return dicts and state_dict keys:
  SwinTransformerV2               model.py:970-1129
  SwinFusion                      model.py:1131-1555
  Transformer_Net_Cross_Attention model.py:341-552
plus the build-defined 3D composite of SURVEY §8d C4 (SwinCrossmodal3D).

3D lift: pass `volume_size` (e.g. 96) in kwargs; inputs become (B, D, H, W) volumes, the
patch-embed conv becomes Conv3d(k=s=patch) and every window is (ws, ws, ws).  Activations
are kept channels-last (B, *spatial, C) end to end: the reference's patch_unembed / patch_embed
transposes around its convolutions (model.py:1396-1482) do not exist here; its convs run on the
channels-last HIP conv kernel with the LeakyReLU fused.
"""
import os
from abc import ABC, abstractmethod

import torch
import torch.nn as nn
import torch.nn.functional as F

from .modules.crossmodal_transformer import TransformerEncoder
from .modules.swin_v2_module import BasicLayer, PatchEmbed, PatchMerging
from .modules.swinfusion_module import (RSTB, CRSTB, PatchEmbed_fusion, PatchUnEmbed, Upsample, UpsampleOneStep,
                                        Cross_BasicLayer, conv_tokens)
from .modules._common import trunc_normal_
from .functional import SplitKLinear, layer_norm


class BaseModel(nn.Module, ABC):
    """Checkpoint helpers shared by the models (model.py:20-151)."""

    def __init__(self):
        super().__init__()
        self.best_loss = 1000000
        self.best_AUROC = 0

    @abstractmethod
    def forward(self, x):
        pass

    @property
    def device(self):
        return next(self.parameters()).device

    def load_partial_state_dict(self, state_dict, load_cls_embedding):
        """Copy matching entries; skip cls embeddings on request and position tensors of a
        different shape (model.py:90-108)."""
        print('loading parameters onto new model...')
        own = self.state_dict()
        loaded = {k: False for k in own}
        for name, param in state_dict.items():
            if name not in own:
                print('notice: {} is not part of new model and was not loaded.'.format(name))
                continue
            if 'cls_embedding' in name and not load_cls_embedding:
                continue
            if 'position' in name and param.shape != own[name].shape:
                print('debug line above')
                continue
            own[name].copy_(param.data)
            loaded[name] = True
        for name, ok in loaded.items():
            if not ok:
                print('notice: named parameter - {} is randomly initialized'.format(name))

    def save_checkpoint(self, directory, title, epoch, loss, AUROC, optimizer=None, schedule=None):
        """Write <title>_last_epoch.pth and the best-loss / best-AUROC copies (model.py:111-151)."""
        os.makedirs(directory, exist_ok=True)
        ckpt = {'model_state_dict': self.state_dict(),
                'optimizer_state_dict': optimizer.state_dict() if optimizer is not None else None,
                'epoch': epoch, 'loss_value': loss}
        if AUROC is not None:
            ckpt['AUROC'] = AUROC
        if schedule is not None:
            ckpt['schedule_state_dict'] = schedule.state_dict()
            ckpt['lr'] = schedule.get_last_lr()[0]
        if hasattr(self, 'loaded_model_weights_path'):
            ckpt['loaded_model_weights_path'] = self.loaded_model_weights_path
        torch.save(ckpt, os.path.join(directory, f"{title}_last_epoch.pth"))
        if AUROC is None and self.best_loss > loss:
            self.best_loss = loss
            torch.save(ckpt, os.path.join(directory, f"{title}_BEST_val_loss.pth"))
            print('updating best saved model...')
        if AUROC is not None and self.best_AUROC < AUROC:
            self.best_AUROC = AUROC
            torch.save(ckpt, os.path.join(directory, f"{title}_BEST_val_AUROC.pth"))
            print('updating best saved model...')


def _init_linear_ln(m):
    if isinstance(m, nn.Linear):
        trunc_normal_(m.weight, std=.02)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.LayerNorm):
        nn.init.constant_(m.bias, 0)
        nn.init.constant_(m.weight, 1.0)


class SwinTransformerV2(BaseModel):
    """Single-modality Swin-V2 classifier (model.py:970-1129).

    kwargs read as in the reference: fine_tune_task, size_of_model, swin_embed_dim, drop_rate,
    attn_drop_rate, mlp_ratio, drop_path_rate, intermediate_vec (image side), patch_size,
    window_size, no_init_weights; plus the build's volume_size for the 3D lift.
    """

    def __init__(self, **kwargs):
        super().__init__()
        self.task = kwargs.get('fine_tune_task')
        self.num_classes = 1
        self.size_of_model = kwargs.get('size_of_model')
        if self.size_of_model == 'small':
            self.depths, self.num_heads_swin = [2], [3]
        elif self.size_of_model == 'medium':
            self.depths, self.num_heads_swin = [2, 2], [3, 6]
        else:
            self.depths, self.num_heads_swin = [2, 2, 6], [3, 6, 12]
        self.num_layers = len(self.depths)
        self.embed_dim = kwargs.get('swin_embed_dim')
        self.ape = False
        self.qkv_bias = True
        self.patch_norm = True
        self.use_checkpoint = bool(kwargs.get('use_checkpoint', False))
        self.num_features = int(self.embed_dim * 2 ** (self.num_layers - 1))
        self.drop_rate = kwargs.get('drop_rate')
        self.attn_drop_rate = kwargs.get('attn_drop_rate')
        self.mlp_ratio = kwargs.get('mlp_ratio')
        self.drop_path_rate = kwargs.get('drop_path_rate')
        self.volume_size = kwargs.get('volume_size')
        side = self.volume_size or kwargs.get('intermediate_vec')
        self.img_size_w = self.img_size_h = side
        self.patch_size = kwargs.get('patch_size')
        self.in_chans = 1
        self.norm_layer = nn.LayerNorm
        self.pretrained_window_sizes = [0, 0, 0, 0]
        self.window_size = kwargs.get('window_size')
        self.patch_embed = PatchEmbed(img_size_w=self.img_size_w, img_size_h=self.img_size_h,
                                      patch_size=self.patch_size, in_chans=self.in_chans, embed_dim=self.embed_dim,
                                      norm_layer=self.norm_layer if self.patch_norm else None,
                                      img_size_d=self.volume_size)
        res = self.patch_embed.patches_resolution
        self.patches_resolution = res
        if self.ape:
            self.absolute_pos_embed = nn.Parameter(torch.zeros(1, self.patch_embed.num_patches, self.embed_dim))
            trunc_normal_(self.absolute_pos_embed, std=.02)
        self.pos_drop = nn.Dropout(p=self.drop_rate)
        dpr = [x.item() for x in torch.linspace(0, self.drop_path_rate, sum(self.depths))]
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            layer_res = tuple(r // (2 ** i) for r in res)
            self.layers.append(BasicLayer(
                dim=int(self.embed_dim * 2 ** i), input_resolution=layer_res, depth=self.depths[i],
                num_heads_swin=self.num_heads_swin[i], window_size=self.window_size, mlp_ratio=self.mlp_ratio,
                qkv_bias=self.qkv_bias, drop=self.drop_rate, attn_drop=self.attn_drop_rate,
                drop_path=dpr[sum(self.depths[:i]):sum(self.depths[:i + 1])], norm_layer=self.norm_layer,
                downsample=PatchMerging if (i < self.num_layers - 1) else None,
                use_checkpoint=self.use_checkpoint, pretrained_window_size=self.pretrained_window_sizes[i]))
        self.norm = self.norm_layer(self.num_features)
        self.avgpool = nn.AdaptiveAvgPool1d(1)
        self.head = nn.Linear(self.num_features, self.num_classes) if self.num_classes > 0 else nn.Identity()
        if kwargs.get('no_init_weights') is False:
            self.apply(_init_linear_ln)
        for bly in self.layers:
            bly._init_respostnorm()

    @torch.jit.ignore
    def no_weight_decay(self):
        return {'absolute_pos_embed'}

    @torch.jit.ignore
    def no_weight_decay_keywords(self):
        return {"cpb_mlp", "logit_scale", 'relative_position_bias_table'}

    def forward_features(self, x):
        x = self.patch_embed(x)
        if self.ape:
            x = x + self.absolute_pos_embed
        x = self.pos_drop(x)
        for layer in self.layers:
            x = layer(x)
        x = layer_norm(x, self.norm)
        return x.mean(dim=1)   # == AdaptiveAvgPool1d(1) over tokens, flattened

    def forward(self, x):
        x = self.forward_features(x.unsqueeze(dim=1))
        return {self.task: self.head(x)}


class SwinFusion(BaseModel):
    """Two-modality SwinIR-style fusion trunk + Swin-V2 head (model.py:1131-1555).

    Forward (A, B): (B, 84, 84) pairs in 2D, (B, D, H, W) volumes in the 3D lift
    (volume_size kwarg).  Returns {fine_tune_task: logits (B, 1)}.
    """

    def __init__(self, img_size=84, patch_size=7, in_chans=1,
                 embed_dim=12, Ex_depths=[6, 6], Fusion_depths=[2, 2, 2], Re_depths=[6, 6],
                 Ex_num_heads=[6, 6], Fusion_num_heads=[6, 6, 6], Re_num_heads=[6, 6],
                 window_size=6, mlp_ratio=4., qkv_bias=True, qk_scale=None,
                 drop_rate=0.8, attn_drop_rate=0.8, drop_path_rate=0.1,
                 norm_layer=nn.LayerNorm, ape=False, patch_norm=True,
                 use_checkpoint=False, upscale=2, img_range=1., upsampler='', resi_connection='1conv',
                 **kwargs):
        super().__init__()
        self.task = kwargs.get('fine_tune_task')
        self.volume_size = kwargs.get('volume_size')
        self.nd = 3 if self.volume_size else 2
        if self.volume_size:
            img_size = self.volume_size
        num_out_ch = in_chans
        num_feat = 64
        self.img_range = img_range
        half = int(embed_dim / 2)
        # non-persistent buffers: they follow .to(device) (no per-step host->device copy, graph
        # capturable) and stay out of the state_dict, like the reference's plain attributes
        if in_chans == 3 or in_chans == 6:
            self.register_buffer('mean', torch.Tensor((0.4488, 0.4371, 0.4040)).view(1, 3, 1, 1), persistent=False)
            self.register_buffer('mean_in', torch.Tensor((0.4488, 0.4371, 0.4040) * 2).view(1, 6, 1, 1),
                                 persistent=False)
        else:
            self.register_buffer('mean', torch.zeros(1), persistent=False)
        self.upscale = upscale
        self.upsampler = upsampler
        self.window_size = window_size
        # Swin-V2 head: explicit args win over the outer kwargs exactly as in model.py:1185-1191
        head_kw = dict(kwargs)
        head_kw.update(patch_size=patch_size, window_size=window_size, mlp_ratio=4., drop_rate=0.,
                       attn_drop_rate=0., drop_path_rate=0.1)
        if self.volume_size:
            head_kw['volume_size'] = self.volume_size
        self.swin = SwinTransformerV2(img_size_w=img_size, img_size_h=img_size, in_chans=1, num_classes=1,
                                      embed_dim=12, depths=[2, 2, 6], num_heads_swin=[3, 6, 12], qkv_bias=True,
                                      norm_layer=nn.LayerNorm, ape=False, patch_norm=True,
                                      pretrained_window_sizes=[0, 0, 0, 0], **head_kw)
        conv = nn.Conv2d if self.nd == 2 else nn.Conv3d
        self.conv_first1_A = conv(in_chans, half, 3, 1, 1)
        self.conv_first1_B = conv(in_chans, half, 3, 1, 1)
        self.conv_first2_A = conv(half, embed_dim, 3, 1, 1)
        self.conv_first2_B = conv(half, half, 3, 1, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        self.Ex_num_layers = len(Ex_depths)
        self.Fusion_num_layers = len(Fusion_depths)
        self.Re_num_layers = len(Re_depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.num_features = embed_dim
        self.mlp_ratio = mlp_ratio
        self.patch_embed = PatchEmbed_fusion(img_size=img_size, patch_size=patch_size, in_chans=embed_dim,
                                             embed_dim=embed_dim, norm_layer=norm_layer if patch_norm else None)
        pr = self.patch_embed.patches_resolution
        if self.nd == 3:
            pr = [img_size // patch_size] * 3
        self.patches_resolution = pr
        self.patch_unembed = PatchUnEmbed(img_size=img_size, patch_size=patch_size, in_chans=embed_dim,
                                          embed_dim=embed_dim, norm_layer=norm_layer if patch_norm else None)
        self.softmax = nn.Softmax(dim=0)
        if self.ape:
            self.absolute_pos_embed = nn.Parameter(torch.zeros(1, self.patch_embed.num_patches, embed_dim))
            trunc_normal_(self.absolute_pos_embed, std=.02)
        self.pos_drop = nn.Dropout(p=drop_rate)
        res = tuple(pr)

        def dpr(depths):
            return [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]

        def group(cls, depths, heads, i, rates):
            return cls(dim=embed_dim, input_resolution=res, depth=depths[i], num_heads=heads[i],
                       window_size=window_size, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                       drop=drop_rate, attn_drop=attn_drop_rate,
                       drop_path=rates[sum(depths[:i]):sum(depths[:i + 1])], norm_layer=norm_layer,
                       downsample=None, use_checkpoint=use_checkpoint, img_size=img_size, patch_size=patch_size,
                       resi_connection=resi_connection)

        r_ex, r_fu, r_re = dpr(Ex_depths), dpr(Fusion_depths), dpr(Re_depths)
        self.layers_Ex_A = nn.ModuleList([group(RSTB, Ex_depths, Ex_num_heads, i, r_ex)
                                          for i in range(self.Ex_num_layers)])
        self.norm_Ex_A = norm_layer(self.num_features)
        self.layers_Ex_B = nn.ModuleList([group(RSTB, Ex_depths, Ex_num_heads, i, r_ex)
                                          for i in range(self.Ex_num_layers)])
        self.norm_Ex_B = norm_layer(self.num_features)
        self.layers_Fusion = nn.ModuleList([group(CRSTB, Fusion_depths, Fusion_num_heads, i, r_fu)
                                            for i in range(self.Fusion_num_layers)])
        self.norm_Fusion_A = norm_layer(self.num_features)
        self.norm_Fusion_B = norm_layer(self.num_features)
        self.layers_Re = nn.ModuleList([group(RSTB, Re_depths, Re_num_heads, i, r_re)
                                        for i in range(self.Re_num_layers)])
        self.norm_Re = norm_layer(self.num_features)
        if resi_connection == '1conv':
            self.conv_after_body_Ex_A = conv(embed_dim, embed_dim, 3, 1, 1)
            self.conv_after_body_Fusion = conv(2 * embed_dim, embed_dim, 3, 1, 1)
            self.conv_after_body_Re = conv(embed_dim, embed_dim, 3, 1, 1)
        elif resi_connection == '3conv':
            self.conv_after_body = nn.Sequential(conv(embed_dim, embed_dim // 4, 3, 1, 1),
                                                 nn.LeakyReLU(negative_slope=0.2, inplace=True),
                                                 conv(embed_dim // 4, embed_dim // 4, 1, 1, 0),
                                                 nn.LeakyReLU(negative_slope=0.2, inplace=True),
                                                 conv(embed_dim // 4, embed_dim, 3, 1, 1))
        if self.upsampler == 'pixelshuffle':
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, num_feat, 3, 1, 1),
                                                      nn.LeakyReLU(inplace=True))
            self.upsample = Upsample(upscale, num_feat)
            self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        elif self.upsampler == 'pixelshuffledirect':
            self.upsample = UpsampleOneStep(upscale, embed_dim, num_out_ch, (pr[0], pr[1]))
        elif self.upsampler == 'nearest+conv':
            assert self.upscale == 4, 'only support x4 now.'
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, num_feat, 3, 1, 1),
                                                      nn.LeakyReLU(inplace=True))
            self.conv_up1 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_up2 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_hr = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
            self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        else:
            self.conv_last1 = conv(embed_dim, half, 3, 1, 1)
            self.conv_last2 = conv(half, int(half / 2), 3, 1, 1)
            self.conv_last3 = conv(int(half / 2), num_out_ch, 3, 1, 1)
        self.apply(_init_linear_ln)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {'absolute_pos_embed'}

    @torch.jit.ignore
    def no_weight_decay_keywords(self):
        return {'relative_position_bias_table'}

    def check_image_size(self, x):
        """Reflect-pad the spatial dims of a (B, 1, *spatial) input to multiples of the window
        (model.py:1389-1394)."""
        pads = []
        for n in reversed(x.shape[2:]):
            pads += [0, (self.window_size - n % self.window_size) % self.window_size]
        if any(pads):
            x = F.pad(x, pads, 'reflect')
        return x

    # token helpers: channels-last maps (B, *spatial, C) <-> tokens (B, L, C) are free reshapes
    def _embed(self, x_cl):
        B, C = x_cl.shape[0], x_cl.shape[-1]
        t = x_cl.reshape(B, -1, C)
        if self.patch_embed.norm is not None:
            t = layer_norm(t, self.patch_embed.norm)
        if self.ape:
            t = t + self.absolute_pos_embed
        return self.pos_drop(t)

    @staticmethod
    def _unembed(t, x_size):
        return t.reshape(t.shape[0], *x_size, t.shape[-1])

    def _extract(self, x_cl, layers, norm):
        x = conv_tokens(self.conv_first1_A, x_cl, 0.2)
        x = conv_tokens(self.conv_first2_A, x, 0.2)
        x_size = tuple(x.shape[1:-1])
        t = self._embed(x)
        for layer in layers:
            t = layer(t, x_size)
        return self._unembed(layer_norm(t, norm), x_size)

    def forward_features_Ex_A(self, x_cl):
        return self._extract(x_cl, self.layers_Ex_A, self.norm_Ex_A)

    def forward_features_Ex_B(self, x_cl):
        # the reference's Ex_B branch reuses the *_A shallow convs (model.py:1414-1415; Q5)
        return self._extract(x_cl, self.layers_Ex_B, self.norm_Ex_B)

    def forward_features_Fusion(self, x_cl, y_cl):
        x_size = tuple(x_cl.shape[1:-1])
        x, y = self._embed(x_cl), self._embed(y_cl)
        for layer in self.layers_Fusion:
            x, y = layer(x, y, x_size)
        x = self._unembed(layer_norm(x, self.norm_Fusion_A), x_size)
        y = self._unembed(layer_norm(y, self.norm_Fusion_B), x_size)
        return conv_tokens(self.conv_after_body_Fusion, torch.cat([x, y], -1), 0.2)

    def forward_features_Re(self, x_cl):
        x_size = tuple(x_cl.shape[1:-1])
        t = self._embed(x_cl)
        for layer in self.layers_Re:
            t = layer(t, x_size)
        x = self._unembed(layer_norm(t, self.norm_Re), x_size)
        x = conv_tokens(self.conv_last1, x, 0.2)
        x = conv_tokens(self.conv_last2, x, 0.2)
        return conv_tokens(self.conv_last3, x, 1.0)

    def forward(self, A, B):
        x = A.unsqueeze(dim=1)
        y = B.unsqueeze(dim=1)
        spatial = tuple(x.shape[2:])
        x = self.check_image_size(x)
        y = self.check_image_size(y)
        mean = self.mean.type_as(x)
        x = (x - mean) * self.img_range
        y = (y - mean) * self.img_range
        # (B, 1, *spatial) is already channels-last with C = 1
        x = x.reshape(x.shape[0], *x.shape[2:], 1)
        y = y.reshape(y.shape[0], *y.shape[2:], 1)
        x = self.forward_features_Ex_A(x)
        y = self.forward_features_Ex_B(y)
        x = self.forward_features_Fusion(x, y)
        x = self.forward_features_Re(x)
        x = x / self.img_range + mean
        crop = tuple(slice(0, n * self.upscale) for n in spatial)
        x = x[(slice(None),) + crop + (0,)]
        return self.swin(x)


class Transformer_Net_Cross_Attention(BaseModel):
    """Crossmodal (low <-> ultra-low frequency fMRI) transformer classifier (model.py:341-552)."""

    def __init__(self, **kwargs):
        super().__init__()
        self.task = kwargs.get('fine_tune_task')
        self.orig_d_l = self.orig_d_u = kwargs.get('intermediate_vec')
        self.d_l = self.d_u = kwargs.get('intermediate_vec')
        self.num_heads_mult = kwargs.get('num_heads_mult')
        self.layers = kwargs.get('nlevels')
        self.attn_dropout = kwargs.get('attn_dropout')
        self.attn_dropout_u = kwargs.get('attn_dropout_u')
        self.relu_dropout = kwargs.get('relu_dropout')
        self.res_dropout = kwargs.get('res_dropout')
        self.out_dropout = kwargs.get('out_dropout')
        self.embed_dropout = kwargs.get('embed_dropout')
        self.attn_mask = kwargs.get('attn_mask')
        self.sequence_length = kwargs.get('sequence_length')
        self.fine_tune_task = kwargs.get('fine_tune_task')
        self.feature_map_gen = kwargs.get('feature_map_gen')
        self.feature_map_size = kwargs.get('feature_map_size')
        self.mixing = kwargs.get('mixing')
        self.concat_method = kwargs.get('concat_method')
        self.fmri_type = kwargs.get('fmri_type')
        combined_dim = self.d_l + self.d_u
        output_dim = 1
        T = self.sequence_length
        if self.feature_map_size == 'different':
            if self.feature_map_gen == 'convolution_ul+l':
                self.proj_l = nn.Conv1d(T, T, kernel_size=1, padding=0, bias=False)
                self.proj_u = nn.Conv1d(T, T // 2, kernel_size=1, padding=0, bias=False)
            elif self.feature_map_gen == 'convolution_ul':
                self.proj_u = nn.Conv1d(T, T // 2, kernel_size=1, padding=0, bias=False)
        elif self.feature_map_size == 'same':
            if self.feature_map_gen == 'convolution_ul+l':
                self.proj_l = nn.Conv1d(T, T, kernel_size=1, padding=0, bias=False)
        self.trans_l_with_u = self.get_network(self_type='lu')
        self.trans_u_with_l = self.get_network(self_type='ul')
        if self.feature_map_size == 'different' or self.fmri_type == 'timeseries_and_frequency':
            self.deconv = nn.ConvTranspose1d(T // 2, T, kernel_size=1, padding=0, bias=False)
        self.trans_mem = self.get_network(self_type='mem', layers=3)
        self.trans_l_mem = self.get_network(self_type='l_mem', layers=3)
        self.trans_u_mem = self.get_network(self_type='u_mem', layers=3)
        self.proj1 = nn.Linear(combined_dim, combined_dim)
        self.proj2 = nn.Linear(combined_dim, combined_dim)
        self.out_layer1 = nn.Linear(combined_dim, combined_dim // 2)
        self.out_layer2 = nn.Linear(combined_dim // 2, output_dim)

    def get_network(self, self_type='lu', layers=-1):
        table = {'ul': (self.d_l, self.attn_dropout), 'lu': (self.d_u, self.attn_dropout_u),
                 'l_mem': (self.d_l, self.attn_dropout), 'u_mem': (self.d_u, self.attn_dropout_u),
                 'mem': (self.d_u * 2, self.attn_dropout)}
        if self_type not in table or self.feature_map_size not in ('same', 'different'):
            raise ValueError("Unknown network type")
        embed_dim, attn_dropout = table[self_type]
        return TransformerEncoder(embed_dim=embed_dim, num_heads_mult=self.num_heads_mult,
                                  layers=max(self.layers, layers), attn_dropout=attn_dropout,
                                  relu_dropout=self.relu_dropout, res_dropout=self.res_dropout,
                                  embed_dropout=self.embed_dropout, attn_mask=self.attn_mask)

    def forward(self, x_l, x_u):
        """x_l, x_u: (B, T, features) -> {'embedding_per_ROIs': (B, d), task: (B, 1)}."""
        drop = lambda t: F.dropout(t, p=self.embed_dropout, training=self.training)  # noqa: E731
        if self.feature_map_size == 'different':
            if self.feature_map_gen == 'convolution_ul+l':
                proj_x_l = self.proj_l(drop(x_l)).transpose(1, 2)
                proj_x_u = self.proj_u(x_u).transpose(1, 2)
            elif self.feature_map_gen == 'convolution_ul':
                proj_x_l = drop(x_l.transpose(1, 2))
                proj_x_u = self.proj_u(x_u).transpose(1, 2)
        elif self.feature_map_size == 'same':
            if self.feature_map_gen == 'no':
                proj_x_l = drop(x_l.transpose(1, 2))
                proj_x_u = x_u.transpose(1, 2)
            elif self.feature_map_gen == 'convolution_ul+l':
                proj_x_l = self.proj_l(drop(x_l)).transpose(1, 2)
                proj_x_u = self.proj_l(x_u).transpose(1, 2)
        proj_x_u = proj_x_u.permute(2, 0, 1)
        proj_x_l = proj_x_l.permute(2, 0, 1)
        h_l_with_us = self.trans_l_with_u(proj_x_l, proj_x_u, proj_x_u)
        h_u_with_ls = self.trans_u_with_l(proj_x_u, proj_x_l, proj_x_l)
        if self.feature_map_size == 'different' or self.fmri_type == 'timeseries_and_frequency':
            h_u_with_ls = self.deconv(h_u_with_ls.transpose(0, 1).float()).transpose(0, 1)
        if self.mixing == 'U2L_and_L2U':
            if self.concat_method == 'concat':
                h_zs = self.trans_mem(torch.cat([h_l_with_us, h_u_with_ls], dim=2))
                out_cls = self.out_layer1(h_zs[-1])
            elif self.concat_method == 'hadamard':
                h_zs = self.trans_l_mem(torch.mul(h_l_with_us, h_u_with_ls))
                out_cls = h_zs[-1]
        elif self.mixing == 'U2L':
            out_cls = self.trans_l_mem(h_l_with_us)[-1]
        elif self.mixing == 'L2U':
            out_cls = self.trans_u_mem(h_u_with_ls)[-1]
        pred = self.out_layer2(out_cls)
        return {'embedding_per_ROIs': out_cls, self.task: pred}


class SwinCrossmodal3D(BaseModel):
    """Build-defined C4 composite (the reference's Func_Struct_Cross,
    model.py:1948-2020, is not instantiable, so its topology is composed from the hot-path modules):

        per modality   PatchEmbed Conv3d(k=s=patch) + LN -> Swin-V2 stage 1 (BasicLayer, 2 blocks,
                       swin heads, window ws; swin_v2_module.py:425-433)
        fusion         Cross_BasicLayer (2 Cross_SwinTransformerBlocks, cross_heads;
                       swinfusion_module.py:698-747)
        to sequences   Linear(embed -> intermediate_vec) per modality: (B, L, d) token sequences
        head           the crossmodal topology of Transformer_Net_Cross_Attention
                       (model.py:489-537: l<-u and u<-l encoders, concat, trans_mem, last token,
                       out_layer1/2; nlevels layers, num_heads_mult heads, causal mask) on the
                       L = (volume / patch)^3 token sequences, feature_map_gen 'no'.
    forward(A, B): two (B, D, H, W) volumes -> {'embedding_per_ROIs', fine_tune_task: (B, 1)}.

    C5: modality B may have its own volume and patch (`volume_size_B`,
    `patch_size_B`; 128^3 fMRI / 8 and 96^3 sMRI / 6 both give 16^3 tokens), and
    `head_dtype='bf16'` runs to_seq + the crossmodal head under bf16 autocast: fp32 master
    weights, bf16 GEMMs and activations, the bf16 MHA kernels on bf16 q/k/v, fp32 LayerNorm and
    softmax.  The Swin front-end (<1% of C5's FLOPs) stays fp32.
    """

    def __init__(self, **kwargs):
        super().__init__()
        self.task = kwargs.get('fine_tune_task')
        self.volume_size = kwargs.get('volume_size') or 96
        self.patch_size = kwargs.get('patch_size') or 8
        self.embed_dim = kwargs.get('swin_embed_dim') or 12
        ws = kwargs.get('window_size') or 6
        swin_heads = kwargs.get('swin_heads') or 3
        cross_heads = kwargs.get('cross_heads') or 6
        depth = kwargs.get('swin_depth') or 2
        mlp_ratio = kwargs.get('mlp_ratio') or 4.0
        d = kwargs.get('intermediate_vec') or 84
        use_ckpt = bool(kwargs.get('use_checkpoint', False))
        V, P, E = self.volume_size, self.patch_size, self.embed_dim
        VB = kwargs.get('volume_size_B') or V
        PB = kwargs.get('patch_size_B') or P
        hd = kwargs.get('head_dtype') or 'fp32'
        if hd not in ('fp32', 'bf16'):
            raise ValueError(f"head_dtype must be 'fp32' or 'bf16', got {hd!r}")
        self.head_dtype = torch.bfloat16 if hd == 'bf16' else torch.float32

        def embed(v, p):
            return PatchEmbed(img_size_w=v, img_size_h=v, patch_size=p, in_chans=1, embed_dim=E,
                              norm_layer=nn.LayerNorm, img_size_d=v)

        self.patch_embed_A, self.patch_embed_B = embed(V, P), embed(VB, PB)
        res = tuple(self.patch_embed_A.patches_resolution)
        if tuple(self.patch_embed_B.patches_resolution) != res:
            raise ValueError(f"modality token grids differ: {res} vs {tuple(self.patch_embed_B.patches_resolution)} "
                             "(volume_size / patch_size must match volume_size_B / patch_size_B)")
        self.patches_resolution = res

        def stage():
            return BasicLayer(dim=E, input_resolution=res, depth=depth, num_heads_swin=swin_heads, window_size=ws,
                              mlp_ratio=mlp_ratio, qkv_bias=True, drop=0.0, attn_drop=0.0, drop_path=0.0,
                              norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=use_ckpt)

        self.swin_A, self.swin_B = stage(), stage()
        self.cross = Cross_BasicLayer(dim=E, input_resolution=res, depth=depth, num_heads=cross_heads, window_size=ws,
                                      mlp_ratio=mlp_ratio, use_checkpoint=use_ckpt)
        self.to_seq_A = SplitKLinear(E, d)
        self.to_seq_B = SplitKLinear(E, d)
        head_kw = dict(kwargs)
        head_kw.update(intermediate_vec=d, feature_map_gen='no', feature_map_size='same',
                       sequence_length=int(res[0] * res[1] * res[2]))
        self.crossmodal = Transformer_Net_Cross_Attention(**head_kw)
        for bly in (self.swin_A, self.swin_B):
            bly._init_respostnorm()

    def forward(self, A, B):
        x = self.swin_A(self.patch_embed_A(A.unsqueeze(1)))
        y = self.swin_B(self.patch_embed_B(B.unsqueeze(1)))
        x, y = self.cross(x, y, self.patches_resolution)
        if self.head_dtype == torch.float32:
            return self.crossmodal(self.to_seq_A(x), self.to_seq_B(y))
        with torch.autocast(device_type="cuda", dtype=self.head_dtype):
            out = self.crossmodal(self.to_seq_A(x), self.to_seq_B(y))
        return {k: (v.float() if torch.is_tensor(v) else v) for k, v in out.items()}

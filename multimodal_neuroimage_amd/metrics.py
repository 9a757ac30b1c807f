"""Validation metrics of the training driver (metrics.py + loss_writer.py:75-128 of the reference).

Per subject the writer averages sigmoid(logit) over that subject's predictions; a set's metrics
are then computed over subjects with scikit-learn, the library the reference calls:
  classification  Balanced_Accuracy, Regular_Accuracy (prediction > 0.5), AUROC, and the
                  ROC-curve operating point with the largest G-mean: best_bal_acc, best_threshold,
                  gmean, specificity, sensitivity, f1_score (the test set uses the stored
                  validation threshold instead)
  regression      MAE, MSE, NMSE, R2_score
The subject records of all ranks are gathered before the metrics (the reference computes them
per rank on that rank's shard).
"""
import numpy as np
from sklearn.metrics import balanced_accuracy_score, f1_score, r2_score, recall_score, roc_auc_score, roc_curve


def classification_metrics(truth, pred, name, val_threshold):
    """{name_metric: value} for one set, as Writer.accuracy_summary reports them."""
    truth = np.asarray(truth)
    pred = np.asarray(pred, dtype=np.float64)
    out = {
        f"{name}_Balanced_Accuracy": balanced_accuracy_score(truth, pred > 0.5),
        f"{name}_Regular_Accuracy": float(np.mean(truth == (pred > 0.5))),
        f"{name}_AUROC": roc_auc_score(truth, pred),
    }
    if name == "test":
        thr = val_threshold
        hard = pred > thr
        tpr = recall_score(truth, hard, pos_label=1)
        tnr = recall_score(truth, hard, pos_label=0)
        gmean, spec, sens = np.sqrt(tpr * tnr), tnr, tpr
    else:
        fpr, tpr_c, thresholds = roc_curve(truth, pred)
        g = np.sqrt(tpr_c * (1 - fpr))
        ix = int(np.argmax(g))
        thr, gmean, spec, sens = thresholds[ix], g[ix], 1 - fpr[ix], tpr_c[ix]
        hard = pred > thr
    out[f"{name}_best_bal_acc"] = balanced_accuracy_score(truth, hard)
    out[f"{name}_best_threshold"] = float(thr)
    out[f"{name}_gmean"] = float(gmean)
    out[f"{name}_specificity"] = float(spec)
    out[f"{name}_sensitivity"] = float(sens)
    out[f"{name}_f1_score"] = f1_score(truth, hard)
    return {k: float(v) for k, v in out.items()}


def regression_metrics(truth, pred, name):
    truth = np.asarray(truth, dtype=np.float64)
    pred = np.asarray(pred, dtype=np.float64)
    return {f"{name}_MAE": float(np.mean(np.abs(pred - truth))),
            f"{name}_MSE": float(np.mean((pred - truth) ** 2)),
            f"{name}_NMSE": float(np.mean((pred - truth) ** 2 / truth ** 2)),
            f"{name}_R2_score": float(r2_score(truth, pred))}

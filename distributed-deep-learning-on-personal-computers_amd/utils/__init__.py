from .metrics import (DeviceMeter, RunLogger, StepTimer, confusion_matrix, dump_pngs,
                      iou_per_class)

__all__ = ["DeviceMeter", "RunLogger", "StepTimer", "dump_pngs", "iou_per_class",
           "confusion_matrix"]

#!/usr/bin/env python3
"""Training entry point with the flags of the reference's scripts/train.py (:39-188).

    python tools/train.py --data processed_data.pkl --embedding_dim 32 --batch_size 1024
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/train.py \
        --data ... --distributed_strategy mirrored

CLI defaults are the reference CLI's (embedding_dim 64, cross_layers 1, batch_size 2048, epochs 5,
ctr_weight 0.2, hard/random negatives 20/30 — note they differ from the ModelConfig defaults,
SURVEY §5). Negative-sampling flags are accepted and stored but, as in the reference, unused.
"""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import recsys_amd  # noqa: E402

logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
logger = logging.getLogger(__name__)


def main():
    p = argparse.ArgumentParser(description="Train Enterprise Recommendation System (MI355X)",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--data", type=str, required=True, help="Path to preprocessed data pickle file")
    p.add_argument("--output_dir", type=str, default="./outputs/models/experiment_001")
    p.add_argument("--embedding_dim", type=int, default=64)
    p.add_argument("--cross_layers", type=int, default=1)
    p.add_argument("--batch_size", type=int, default=2048)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--learning_rate", type=float, default=0.001)
    p.add_argument("--negative_sampling", choices=["random", "hard", "mixed"], default="mixed")
    p.add_argument("--num_hard_negatives", type=int, default=20)
    p.add_argument("--num_random_negatives", type=int, default=30)
    p.add_argument("--ctr_weight", type=float, default=0.2)
    p.add_argument("--rating_weight", type=float, default=0.2)
    p.add_argument("--distributed_strategy", choices=["none", "mirrored", "multi_worker"], default="none")
    p.add_argument("--use_wandb", action="store_true", help="accepted for compatibility; ignored")
    args = p.parse_args()

    config = recsys_amd.ModelConfig(
        embedding_dim=args.embedding_dim, cross_layers=args.cross_layers, batch_size=args.batch_size,
        epochs_retrieval=args.epochs, learning_rate_retrieval=args.learning_rate,
        negative_sampling_strategy=args.negative_sampling, num_hard_negatives=args.num_hard_negatives,
        num_random_negatives=args.num_random_negatives, ctr_weight=args.ctr_weight,
        rating_weight=args.rating_weight, distributed_strategy=args.distributed_strategy)
    logger.info("=" * 80)
    logger.info("TRAINING CONFIGURATION:")
    for k, v in config.to_dict().items():
        logger.info(f"  {k}: {v}")
    logger.info("=" * 80)
    trainer = recsys_amd.ProductionTrainer(config, args.output_dir)
    try:
        trainer.train(args.data)
        logger.info("Training completed successfully! Artifacts saved to: %s", args.output_dir)
    except KeyboardInterrupt:
        logger.warning("Training interrupted by user")
        sys.exit(1)
    except Exception as e:  # same contract as scripts/train.py:175-179
        logger.error(f"Training failed: {e}")
        import traceback
        traceback.print_exc()
        sys.exit(1)


if __name__ == "__main__":
    main()

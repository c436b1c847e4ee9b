"""Trainer-side modules of the reference's src/main (loss, schedule, optimizer, trainer)."""

"""Reference-compatible import path: ``from model import resnet``."""
